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


def _sources():
    files = sorted(glob.glob(os.path.join(JAVA, "**", "*.java"), recursive=True))
    assert len(files) >= 4
    return files


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


def _package_has(pkg, name):
    rel = os.path.join(*pkg.split("."), name + ".java")
    return bool(glob.glob(os.path.join(REF, "**", "src", "main", "java", rel), recursive=True)) or os.path.exists(
        os.path.join(JAVA, rel))


@pytest.mark.parametrize("path", _sources() if os.path.isdir(REF) else [], ids=os.path.basename)
def test_imports_resolve(path):
    src = open(path).read()
    pkg = _package(src)
    assert path.endswith(os.path.join(*pkg.split("."), os.path.basename(path))), "file sits in its package dir"
    imported = set()
    for static, name in re.findall(r"^import\s+(static\s+)?([\w.]+);", src, re.M):
        if name.startswith(("java.", "javax.", "io.netty.")):
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
        assert _package_has(pkg, name), f"{os.path.basename(path)}: {name} is not a class of {pkg}"


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
