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


def test_jni_shim_compiles_against_the_jni_calls_it_makes():
    """gcc -fsyntax-only over jni/gwo_jni.c with tests/jni_stub/jni.h (the JNIEnv functions the shim uses, JDK
    signatures): catches type and arity errors in code that cannot be built here."""
    import shutil
    import subprocess
    import pytest
    if not shutil.which("gcc"):
        pytest.skip("no gcc")
    r = subprocess.run(["gcc", "-fsyntax-only", "-Wall", "-Wextra", "-Werror", "-std=c11",
                        "-I" + os.path.join(ROOT, "tests", "jni_stub"), "-I" + os.path.join(ROOT, "include"),
                        os.path.join(ROOT, "jni", "gwo_jni.c")], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_operator_emits_after_sync_and_reads_max_parallelism_from_the_task():
    """GpuWindowOperator: emitFired completes a running fire (gwo_wait_fires) before counting rows and drains into buffers
    allocated once; the number of key groups is the task's (getMaxNumberOfParallelSubtasks), not ExecutionConfig's;
    the value dtype comes from the aggregate descriptor."""
    op = open(os.path.join(PKG, "GpuWindowOperator.java")).read()
    body = op[op.index("private void emitFired()"):op.index("private String[] keyStrings(")]
    assert body.index("GwoNative.waitFires(handle)") < body.index("GwoNative.outputCount(handle)")
    assert "direct(" not in body.replace("sideKeys = direct(", "").replace("sideTs = direct(", "") \
        .replace("sideValues = direct(", "")
    assert "getRuntimeContext().getMaxNumberOfParallelSubtasks()" in op
    assert "spec.maxParallelism" not in op
    win = open(os.path.join(PKG, "GpuWindows.java")).read()
    assert "spec.valueDtype = fn.valueDtype" in win and "getExecutionConfig().getMaxParallelism" not in win


def test_jni_shim_argument_checks_run_against_a_fake_jvm(tmp_path):
    """jni/gwo_jni.c executed (tests/jni_stub/harness.c: a fake JNIEnv and fake library entry points): the heap-state
    export refuses a null or short keyGroupOffsets array and the import a null byte[] with IllegalArgumentException,
    before the library is reached; well-formed calls reach it (the round-3 advisor's finding)."""
    import shutil
    import subprocess
    import pytest
    if not shutil.which("gcc"):
        pytest.skip("no gcc")
    exe = tmp_path / "harness"
    r = subprocess.run(["gcc", "-std=c11", "-Wall", "-Wno-unused-function", "-I" + os.path.join(ROOT, "tests", "jni_stub"),
                        "-I" + os.path.join(ROOT, "include"), os.path.join(ROOT, "tests", "jni_stub", "harness.c"),
                        # entry points no case reaches stay unresolved (the fake library defines only what is called)
                        "-Wl,--unresolved-symbols=ignore-all", "-o", str(exe)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    out = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split("\n")
    got = {line.split()[0]: line.split()[1:] for line in out if line}
    iae = "java/lang/IllegalArgumentException"
    assert got["export_null_offsets"] == [iae, "0"]
    assert got["export_short_offsets"] == [iae, "0"]
    assert got["export_ok"] == ["-", "2"]          # counting call + writing call
    assert got["export_ok_len"] == ["16", "wm", "42", "last_offset", "7"]
    assert got["import_null_data"] == [iae, "0"]
    assert got["import_ok"] == ["-", "1"]
    assert got["register_null"] == [iae, "0"]
    assert got["register_ok"] == ["-", "1"]
