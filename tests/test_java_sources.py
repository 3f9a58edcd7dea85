"""CPU: the committed Java side of the drop-in boundary (native/java/**) is consistent with the
reference it plugs into, without a JDK (none exists in this image):

* every import resolves — to java.*/javax.*, to Netty (io.netty.*, a Maven dependency the reference
  declares, pom.xml), to a class file under /root/reference/**/src/main/java, or to a class of
  native/java itself; a nested-class or static-member import resolves to its enclosing file;
* every class the sources use from their own package (new X, instanceof X, X.member, implements X)
  exists in that package, in the reference or in native/java;
* GpuIntHash declares every method of IntHash (circe-checksum/.../checksum/IntHash.java:23-35) with
  the same parameter types;
* each reference member the sources rely on is declared where they expect it (the loader of
  NativeUtils.java:54-116, the provider chain's capability flags, DigestManager's ledgerId and
  verifyDigestAndReturnData, ByteBufList's accessors).

Skipped when /root/reference is absent (the GPU box)."""
import glob
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
JAVA = os.path.join(ROOT, "native", "java")

pytestmark = pytest.mark.skipif(not os.path.isdir(REF), reason="reference tree not present")

# java.lang types the sources use without an import
JAVA_LANG = {"String", "Object", "Throwable", "Exception", "RuntimeException", "IllegalArgumentException",
             "IndexOutOfBoundsException", "System", "Math", "Integer", "Long", "Override", "Boolean"}


JAVA_TEST = os.path.join(ROOT, "native", "java-test")


def _sources():
    files = sorted(glob.glob(os.path.join(JAVA, "**", "*.java"), recursive=True))
    assert len(files) >= 4
    # the maintainer-run JUnit test of the batch hooks (native/java-test), resolved the same way
    return files + sorted(glob.glob(os.path.join(JAVA_TEST, "**", "*.java"), recursive=True))


def _package(src):
    return re.search(r"^package\s+([\w.]+);", src, re.M).group(1)


def _ref_class_file(fqcn):
    """The .java file declaring fqcn (or its enclosing class) in the reference or native/java."""
    parts = fqcn.split(".")
    for k in range(len(parts), 1, -1):  # a.b.C.D -> a/b/C/D.java, then a/b/C.java (nested)
        rel = os.path.join(*parts[:k]) + ".java"
        hits = glob.glob(os.path.join(REF, "**", "src", "main", "java", rel), recursive=True)
        local = os.path.join(JAVA, rel)
        if hits:
            return hits[0]
        if os.path.exists(local):
            return local
        if not parts[k - 1][:1].isupper():
            break
    return None


def _package_has(pkg, name, tests=False):
    """A class of pkg in the reference's main sources or native/java; with tests, also the reference's
    test sources (the JUnit tests under native/java-test sit beside them)."""
    rel = os.path.join(*pkg.split("."), name + ".java")
    trees = ("main", "test") if tests else ("main",)
    return any(glob.glob(os.path.join(REF, "**", "src", t, "java", rel), recursive=True) for t in trees) or \
        os.path.exists(os.path.join(JAVA, rel))


@pytest.mark.parametrize("path", _sources() if os.path.isdir(REF) else [], ids=os.path.basename)
def test_imports_resolve(path):
    src = open(path).read()
    pkg = _package(src)
    assert path.endswith(os.path.join(*pkg.split("."), os.path.basename(path))), "file sits in its package dir"
    imported = set()
    for static, name in re.findall(r"^import\s+(static\s+)?([\w.]+);", src, re.M):
        if name.startswith(("java.", "javax.", "io.netty.", "org.junit.")):
            imported.add(name.rsplit(".", 1)[1])
            continue
        fq = name.rsplit(".", 1)[0] if static else name
        assert _ref_class_file(fq), f"{os.path.basename(path)}: import {name} resolves to no class"
        imported.add(name.rsplit(".", 1)[1])
    body = re.sub(r"/\*.*?\*/|//[^\n]*", "", src, flags=re.S)
    used = set(re.findall(r"\b(?:new|instanceof|implements|extends)\s+([A-Z]\w*)", body))
    used |= set(re.findall(r"(?<![\w.])([A-Z]\w*)\.[a-zA-Z_]", body))
    declared = set(re.findall(r"\b(?:class|interface)\s+([A-Z]\w*)", body))
    for name in sorted(used - imported - declared - JAVA_LANG):
        assert _package_has(pkg, name, tests=path.startswith(JAVA_TEST)), \
            f"{os.path.basename(path)}: {name} is not a class of {pkg}"


def test_gpu_int_hash_implements_every_int_hash_method():
    iface = open(_ref_class_file("com.scurrilous.circe.checksum.IntHash")).read()
    methods = re.findall(r"^\s+(\w+)\s+(\w+)\(([^)]*)\);", iface, re.M)
    assert len(methods) == 6  # IntHash.java:23-35
    impl = open(os.path.join(JAVA, "com", "scurrilous", "circe", "checksum", "GpuIntHash.java")).read()
    assert re.search(r"class GpuIntHash implements IntHash\b", impl)
    for ret, name, params in methods:
        types = [p.strip().rsplit(" ", 1)[0] for p in params.split(",") if p.strip()]
        pat = (r"@Override\s+public\s+" + re.escape(ret) + r"\s+" + name + r"\(" +
               r",\s*".join(re.escape(t) + r"\s+\w+" for t in types) + r"\)")
        assert re.search(pat, impl), f"GpuIntHash lacks {ret} {name}({params})"


# (reference class, declaration the Java sources rely on)
MEMBERS = [
    ("org.apache.bookkeeper.common.util.nativelib.NativeUtils", r"public static void loadLibraryFromJar\(String path\)"),
    ("org.apache.bookkeeper.common.util.nativelib.NativeUtils", r"public static String libType\(\)"),
    ("com.scurrilous.circe.crc.Sse42Crc32C", r"public static boolean isSupported\(\)"),
    ("com.scurrilous.circe.crc.Sse42Crc32C", r'loadLibraryFromJar\("/lib/libcirce-checksum\." \+ libType\(\)\)'),
    ("com.scurrilous.circe.checksum.Java9IntHash", r"static final boolean HAS_JAVA9_CRC32C"),
    ("com.scurrilous.circe.checksum.JniIntHash", r"public class JniIntHash implements IntHash"),
    ("com.scurrilous.circe.checksum.Java8IntHash", r"public class Java8IntHash implements IntHash"),
    ("com.scurrilous.circe.checksum.Crc32cIntChecksum", r"private final static IntHash CRC32C_HASH"),
    ("org.apache.bookkeeper.proto.checksum.DigestManager", r"\n    final long ledgerId;"),
    ("org.apache.bookkeeper.proto.checksum.DigestManager", r"public ByteBuf verifyDigestAndReturnData\(long entryId, ByteBuf dataReceived\)"),
    ("org.apache.bookkeeper.proto.checksum.CRC32CDigestManager", r"class CRC32CDigestManager extends DigestManager"),
    ("org.apache.bookkeeper.proto.checksum.CRC32DigestManager", r"class CRC32DigestManager extends DigestManager"),
    ("org.apache.bookkeeper.client.BKException", r"public static class BKDigestMatchException extends BKException"),
    ("org.apache.bookkeeper.util.ByteBufList", r"public ByteBuf getBuffer\(int index\)"),
    ("org.apache.bookkeeper.util.ByteBufList", r"public int size\(\)"),
    ("org.apache.bookkeeper.client.BatchedReadOp", r"lh\.macManager\.verifyDigestAndReturnData\(eId \+ i, buffer\)"),
    # GpuBatchPackager
    ("org.apache.bookkeeper.proto.checksum.DigestManager", r"\n    final boolean useV2Protocol;"),
    ("org.apache.bookkeeper.proto.checksum.DigestManager", r"\n    final int macCodeLength;"),
    ("org.apache.bookkeeper.proto.checksum.DigestManager",
     r"public ReferenceCounted computeDigestAndPackageForSending\(long entryId, long lastAddConfirmed, long length,\s+"
     r"ByteBuf data, byte\[\] masterKey, int flags\)"),
    ("org.apache.bookkeeper.proto.BookieProtoEncoding", r"public static final int SMALL_ENTRY_SIZE_THRESHOLD = 16 \* 1024;"),
    ("org.apache.bookkeeper.proto.BookieProtocol", r"public static int toInt\(byte version, byte opCode, short flags\)"),
    ("org.apache.bookkeeper.proto.BookieProtocol", r"byte CURRENT_PROTOCOL_VERSION = 2;"),
    ("org.apache.bookkeeper.proto.BookieProtocol", r"byte ADDENTRY = 1;"),
    ("org.apache.bookkeeper.proto.BookieProtocol", r"int MASTER_KEY_LENGTH = 20;"),
    ("org.apache.bookkeeper.util.ByteBufList", r"public static ByteBufList get\(ByteBuf b1, ByteBuf b2\)"),
    ("org.apache.bookkeeper.client.LedgerHandle", r"\n    final ClientContext clientCtx;"),
    # native/java-test/.../GpuIntHashTest.java
    ("com.scurrilous.circe.checksum.Crc32cIntChecksum", r"public static int computeChecksum\(ByteBuf payload\)"),
    # native/java-test/.../GpuBatchHooksTest.java
    ("org.apache.bookkeeper.util.ByteBufList", r"public byte\[\] toArray\(\)"),
    ("org.apache.bookkeeper.util.ByteBufList", r"public static ByteBufList get\(\)"),
    ("org.apache.bookkeeper.util.ByteBufList", r"public void add\(ByteBuf buf\)"),
    ("org.apache.bookkeeper.proto.BookieProtocol", r"short FLAG_RECOVERY_ADD = 0x0002;"),
    ("org.apache.bookkeeper.proto.checksum.CRC32CDigestManager",
     r"public CRC32CDigestManager\(long ledgerId, boolean useV2Protocol, ByteBufAllocator allocator\)"),
    ("org.apache.bookkeeper.proto.checksum.CRC32DigestManager",
     r"public CRC32DigestManager\(long ledgerId, boolean useV2Protocol, ByteBufAllocator allocator\)"),
    ("org.apache.bookkeeper.client.ClientContext", r"ByteBufAllocator getByteBufAllocator\(\);"),
    ("org.apache.bookkeeper.client.LedgerFragmentReplicator",
     r"computeDigestAndPackageForSending\(entry\.getEntryId\(\),\s+lh\.getLastAddConfirmed\(\), entry\.getLength\(\),\s+"
     r"Unpooled\.wrappedBuffer\(data, 0, data\.length\),"),
]


@pytest.mark.parametrize("cls,decl", MEMBERS, ids=[f"{c.rsplit('.', 1)[1]}:{i}" for i, (c, _) in enumerate(MEMBERS)])
def test_reference_members_exist(cls, decl):
    path = _ref_class_file(cls)
    assert path and path.startswith(REF), cls
    assert re.search(decl, open(path).read()), f"{cls} lacks {decl}"


def test_integration_doc_names_the_loaded_library():
    """INTEGRATION.md names the library GpuDigest actually loads (the circe jar's /lib/libcirce-checksum)."""
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    gd = open(os.path.join(JAVA, "com", "scurrilous", "circe", "checksum", "GpuDigest.java")).read()
    assert 'loadLibraryFromJar("/lib/libcirce-checksum." + NativeUtils.libType())' in gd
    assert "libbkdigest-jni" not in doc
    assert "GpuProviderChain.select()" in doc and "GpuBatchVerifier.verifiedPrefix" in doc


# ---- GpuBatchVerifier leaves the buffers as verifyDigestAndReturnData does ----
VERIFIER = os.path.join(JAVA, "org", "apache", "bookkeeper", "proto", "checksum", "GpuBatchVerifier.java")
READER_INDEX_SET = "bufList.getBuffer(i).readerIndex(DigestManager.METADATA_LENGTH + dm.macCodeLength);"


def _method_body(src, signature):
    """The text between the braces of the method whose declaration contains `signature`, comments removed."""
    src = re.sub(r"/\*.*?\*/|//[^\n]*", "", src, flags=re.S)
    start = src.index(signature)
    k = src.index("{", start)
    depth = 0
    for j in range(k, len(src)):
        depth += {"{": 1, "}": -1}.get(src[j], 0)
        if depth == 0:
            return src[k + 1:j]
    raise AssertionError("unbalanced braces")


def verifier_problems(src):
    """Why the batched verify hook would leave buffers (or CRC bytes) unlike the reference's loop
    (BatchedReadOp.java:175-189 -> DigestManager.verifyDigestAndReturnData, DigestManager.java:333-338);
    an empty list when it does not. Source-text checks (no JDK here)."""
    problems = []
    body = _method_body(src, "public static int verifiedPrefix(")
    flat = re.sub(r"\s+", " ", body)
    # 1. the GPU route only for buffers nothing has been read from: the reference CRCs absolute
    #    offsets of memoryAddress() (DigestManager.java:62-64,236-239) and reads ids at readerIndex
    if not re.search(r"direct = [^;]*\.hasMemoryAddress\(\) && \w+\.readerIndex\(\) == 0;", flat):
        problems.append("no readerIndex() == 0 guard on the GPU route")
    if re.search(r"memoryAddress\(\) \+ \w+\.readerIndex\(\)", flat):
        problems.append("frame address offset by readerIndex (the reference addresses absolute offsets)")
    call = flat.find("GpuDigest.verifyBatch(")
    if call < 0:
        return problems + ["no GpuDigest.verifyBatch call"]
    after = flat[call:]
    # 2. every exit after the library call: the untouched fallback (rc < 0), or the verified count
    #    after the readerIndex loop over exactly the verified prefix (DigestManager.java:336)
    loop = re.search(r"for \(int i = 0; i < verified; i\+\+\) \{ " + re.escape(READER_INDEX_SET) + r" \}", after)
    for m in re.finditer(r"return ([^;]*);", after):
        ret = m.group(1).strip()
        if ret == "serialPrefix(dm, firstEntryId, bufList)":
            if not re.search(r"if \(rc < 0\) \{ $", after[:m.start()]):
                problems.append("a serial fallback after the library call not guarded by rc < 0")
            if loop and m.start() > loop.start():
                problems.append("a serial fallback after buffers were already advanced")
        elif ret == "verified":
            if not loop or loop.end() > m.start():
                problems.append("the verified count is returned without the readerIndex loop before it")
        else:
            problems.append(f"an exit that skips the readerIndex loop: return {ret};")
    if not re.search(r"final int verified = \(int\) rc;", after):
        problems.append("verified is not the library's verified prefix")
    return problems


def test_batch_verifier_leaves_buffers_as_the_reference():
    assert verifier_problems(open(VERIFIER).read()) == []
    # the reference member the loop relies on (package-private, same package)
    dm = open(_ref_class_file("org.apache.bookkeeper.proto.checksum.DigestManager")).read()
    assert re.search(r"\n    final int macCodeLength;", dm)
    assert "dataReceived.readerIndex(METADATA_LENGTH + macCodeLength);" in dm  # DigestManager.java:336


@pytest.mark.parametrize("mutation", [
    ("bufList.getBuffer(i).readerIndex(DigestManager.METADATA_LENGTH + dm.macCodeLength);", ""),  # round-5 code
    ("&& b.readerIndex() == 0", ""),
    ("addrs.writeLongLE(b.memoryAddress());", "addrs.writeLongLE(b.memoryAddress() + b.readerIndex());"),
    ("return verified;", "return (int) rc;"),
    ("i < verified; i++", "i < n; i++"),
])
def test_batch_verifier_check_catches(mutation):
    """The check above fails on each way the hook can diverge (the round-5 hook had the first and third)."""
    src = open(VERIFIER).read()
    old, new = mutation
    assert old in src
    assert verifier_problems(src.replace(old, new)) != []


def test_batch_packager_builds_the_reference_objects():
    """GpuBatchPackager's V2 buffer is built with the statements of computeDigestAndPackageForSendingV2
    (DigestManager.java:126-167) — the same small-entry test, header sizes, allocation, the three
    leading writes and the small/large tail — with the 32-byte header and digest (there
    writeLong x 4 + populateValueAndReset) taken from the library's frame; V3 is
    ByteBufList.get(header buffer of METADATA_LENGTH + macCodeLength, data) (:169-181)."""
    ref = re.sub(r"\s+", " ", _method_body(open(_ref_class_file("org.apache.bookkeeper.proto.checksum.DigestManager")).read(),
                                          "private ReferenceCounted computeDigestAndPackageForSendingV2("))
    src = open(os.path.join(JAVA, "org", "apache", "bookkeeper", "proto", "checksum", "GpuBatchPackager.java")).read()
    ours = re.sub(r"\s+", " ", _method_body(src, "private static ReferenceCounted packageV2("))
    for stmt in ["boolean isSmallEntry = data.readableBytes() < BookieProtoEncoding.SMALL_ENTRY_SIZE_THRESHOLD;",
                 "int payloadSize = data.readableBytes();",
                 "int bufferSize = 4 + headersSize + (isSmallEntry ? payloadSize : 0);",
                 "ByteBuf buf = allocator.buffer(bufferSize, bufferSize);",
                 "buf.writeInt(headersSize + payloadSize);",
                 "buf.writeBytes(masterKey, 0, BookieProtocol.MASTER_KEY_LENGTH);",
                 "buf.writeBytes(data, data.readerIndex(), data.readableBytes()); data.release(); return buf; }",
                 "return ByteBufList.get(buf, data);"]:
        assert stmt in ref, stmt
        assert stmt in ours, stmt
    toint = "BookieProtocol.PacketHeader.toInt( BookieProtocol.CURRENT_PROTOCOL_VERSION, BookieProtocol.ADDENTRY, (short) flags));"
    assert toint in ref and toint in ours
    # headersSize: 4 + master key + METADATA_LENGTH + macCodeLength (frameLen = METADATA_LENGTH + macCodeLength)
    assert "int headersSize = 4 + BookieProtocol.MASTER_KEY_LENGTH + METADATA_LENGTH + macCodeLength;" in ref
    assert "int headersSize = 4 + BookieProtocol.MASTER_KEY_LENGTH + frameLen;" in ours
    body = re.sub(r"\s+", " ", _method_body(src, "public static ReferenceCounted[] packageEntries("))
    assert "final int frameLen = DigestManager.METADATA_LENGTH + dm.macCodeLength;" in body
    assert "ByteBufList.get(Unpooled.buffer(frameLen).writeBytes(frames, i * frameLen, frameLen), data)" in body
    assert "Unpooled.wrappedBuffer(payloads[i], 0, payloads[i].length)" in body  # LedgerFragmentReplicator.java:509
    # the header + digest bytes written in place of writeLong x 4 + populateValueAndReset come after the master key
    assert ours.index("buf.writeBytes(masterKey") < ours.index("buf.writeBytes(frames, at, frameLen);") < ours.index(
        "if (isSmallEntry)")
