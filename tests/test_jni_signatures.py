"""CPU: the JNI shim's exports (native/jni/bkdigest_jni.c) against the Java declarations they bind.

No JDK exists in this image, so the shim is never compiled here; this test pins its C signatures to
a committed restatement of the Java side instead: the six `Sse42Crc32C` natives
(circe-checksum/src/main/java/com/scurrilous/circe/crc/Sse42Crc32C.java:119-129, all `private
static native`) and the `GpuDigest` batch class of INTEGRATION.md §2. Checked: the mangled symbol
(Java_<class with _ for .>_<method>), the JNI return type, JNIEnv* + jclass (static natives) and
the JNI type of every Java parameter, in order."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHIM = os.path.join(ROOT, "native", "jni", "bkdigest_jni.c")

# Java type -> JNI C type (JNI specification, "Primitive Types" / "Reference Types")
JNI = {"boolean": "jboolean", "int": "jint", "long": "jlong", "void": "void", "byte[]": "jbyteArray",
       "int[]": "jintArray", "long[]": "jlongArray", "byte[][]": "jobjectArray", "ByteBuffer": "jobject",
       "String": "jstring"}

# Sse42Crc32C.java:119-129, verbatim method signatures (return type, name, parameter types)
SSE42 = [
    ("boolean", "nativeSupported", []),
    ("int", "nativeArray", ["int", "byte[]", "int", "int", "long"]),
    ("int", "nativeDirectBuffer", ["int", "ByteBuffer", "int", "int", "long"]),
    ("int", "nativeUnsafe", ["int", "long", "long", "long"]),
    ("long", "allocConfig", ["int[]"]),
    ("void", "freeConfig", ["long"]),
]
# INTEGRATION.md §2, com.scurrilous.circe.checksum.GpuDigest
GPU_DIGEST = [
    ("int", "deviceCount", []),
    ("int", "init", ["int"]),
    ("int", "resumeAddress", ["int", "int", "long", "long"]),
    ("int", "resumeArray", ["int", "int", "byte[]", "int", "int"]),
    ("int", "resumeBatch", ["int", "long", "long", "long", "long", "long", "long", "int", "long"]),
    ("long", "verifyBatch", ["int", "long", "long", "boolean", "long", "long", "long", "long"]),
    ("int", "packageBatch", ["int", "long", "long", "long", "long", "long", "long", "long", "long", "long", "long"]),
    ("int", "packageBatchArrays", ["int", "long", "long[]", "long", "long[]", "byte[][]", "long", "long", "long"]),
    ("String", "lastError", []),
]
CLASSES = {"com.scurrilous.circe.crc.Sse42Crc32C": SSE42, "com.scurrilous.circe.checksum.GpuDigest": GPU_DIGEST}


def _exports():
    text = re.sub(r"/\*.*?\*/", "", open(SHIM).read(), flags=re.S)
    out = {}
    for m in re.finditer(r"JNIEXPORT\s+(\w+)\s+JNICALL\s+(Java_\w+)\s*\(([^)]*)\)", text):
        params = [re.sub(r"\s+", " ", p.strip()) for p in m.group(3).split(",")]
        types = [re.match(r"(\w+\s*\**)", p).group(1).replace(" ", "") for p in params]
        out[m.group(2)] = (m.group(1), types)
    return out


def test_every_declared_native_has_its_jni_signature():
    ex = _exports()
    expected = set()
    for cls, methods in CLASSES.items():
        for ret, name, params in methods:
            sym = "Java_" + cls.replace("_", "_1").replace(".", "_") + "_" + name
            expected.add(sym)
            assert sym in ex, f"missing export {sym}"
            got_ret, got_types = ex[sym]
            assert got_ret == JNI[ret], (sym, got_ret)
            assert got_types[:2] == ["JNIEnv*", "jclass"], (sym, got_types)  # static natives
            assert got_types[2:] == [JNI[p] for p in params], (sym, got_types)
    assert set(ex) == expected, f"unexpected exports: {set(ex) - expected}"


@pytest.mark.parametrize("name", [m[1] for m in SSE42])
def test_sse42_natives_match_reference_declarations(name):
    """The committed table restates the reference's Java declarations; where the reference tree is
    present (this container), check the table against the source itself."""
    src = os.path.join("/root/reference", "circe-checksum/src/main/java/com/scurrilous/circe/crc/Sse42Crc32C.java")
    if not os.path.exists(src):
        pytest.skip("reference tree absent (GPU box)")
    text = open(src).read()
    ret, _, params = next(m for m in SSE42 if m[1] == name)
    m = re.search(r"private static native (\S+) " + name + r"\(([^)]*)\);", text)
    assert m, name
    assert m.group(1) == ret
    got = [p.strip().rsplit(" ", 1)[0] for p in m.group(2).split(",") if p.strip()]
    assert got == params


def test_gpu_digest_java_declarations_match_table():
    """native/java/.../GpuDigest.java (the committed Java side of the batch class) declares exactly the
    natives of the table, with the same types, so the shim, the table and the Java source agree."""
    src = os.path.join(ROOT, "native", "java", "com", "scurrilous", "circe", "checksum", "GpuDigest.java")
    text = re.sub(r"/\*.*?\*/", "", open(src).read(), flags=re.S)
    found = {}
    for m in re.finditer(r"public static native (\S+) (\w+)\(([^)]*)\);", text, flags=re.S):
        params = [p.strip().rsplit(" ", 1)[0] for p in m.group(3).split(",") if p.strip()]
        found[m.group(2)] = (m.group(1), params)
    assert found == {name: (ret, params) for ret, name, params in GPU_DIGEST}
