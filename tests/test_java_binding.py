"""CPU: the Java binding (java/.../gpu/GwoNative.java) and the JNI shim (jni/gwo_jni.c) agree with each other and
with include/gwo.h.  There is no JDK in this image, so this checks what can be checked without
one: every native method has exactly one JNI function of the mangled name with the right arity, every C entry
point the shim calls is declared in gwo.h, and the Java constants equal the header's."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "java", "src", "main", "java", "org", "apache", "flink", "streaming", "runtime", "operators",
                   "windowing", "gpu")


def _read(*p):
    return open(os.path.join(ROOT, *p)).read()


def _java_natives():
    src = open(os.path.join(PKG, "GwoNative.java")).read()
    out = {}
    for m in re.finditer(r"static native [\w\[\]<>]+ (\w+)\(([^)]*)\);", src, re.S):
        params = [p for p in m.group(2).split(",") if p.strip()]
        out[m.group(1)] = len(params)
    return out


def _jni_functions():
    src = _read("jni", "gwo_jni.c")
    out = {}
    for m in re.finditer(r"JNICALL JFN\((\w+)\)\(([^)]*)\)", src, re.S):
        out[m.group(1)] = len([p for p in m.group(2).split(",") if p.strip()])
    return out


def test_every_native_has_its_jni_function():
    nat, jni = _java_natives(), _jni_functions()
    assert nat and set(nat) == set(jni)
    for name, n in nat.items():
        assert jni[name] == n + 2, name   # JNIEnv *, jclass


def test_shim_calls_only_declared_entry_points():
    header = _read("include", "gwo.h")
    declared = set(re.findall(r"\b(gwo_\w+)\s*\(", header))
    called = set(re.findall(r"\b(gwo_\w+)\s*\(", _read("jni", "gwo_jni.c")))
    assert called and called <= declared, called - declared


def test_java_constants_match_header():
    java = open(os.path.join(PKG, "GwoNative.java")).read()
    header = _read("include", "gwo.h")
    abi = int(re.search(r"#define GWO_ABI_VERSION (\d+)", header).group(1))
    assert int(re.search(r"ABI_VERSION = (\d+)", java).group(1)) == abi
    enums = dict((k, int(v)) for k, v in re.findall(r"\bGWO_(\w+) = (\d+)", header))
    for name, value in re.findall(r"\b([A-Z0-9_]+) = (\d+)", java):
        if name == "ABI_VERSION":
            continue
        assert enums.get(name) == int(value), name


def test_jni_mangled_class_matches_package():
    src = _read("jni", "gwo_jni.c")
    pkg = re.search(r"^package ([\w.]+);", open(os.path.join(PKG, "GwoNative.java")).read(), re.M).group(1)
    assert "Java_" + pkg.replace(".", "_") + "_GwoNative_##name" in src
