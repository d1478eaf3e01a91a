"""CPU: the C-ABI library loads and exports every symbol include/gwo.h declares."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    src = open(os.path.join(ROOT, "include", "gwo.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(gwo_[a-z_0-9]+)\s*\(", src)))


def test_header_parses():
    names = declared_functions()
    assert "gwo_create" in names and "gwo_submit" in names and "gwo_advance_watermark" in names
    assert len(names) >= 25


def test_library_exports_every_declared_symbol():
    from flink_amd import _native as N
    lib = N.load()
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing


def test_binding_covers_header():
    from flink_amd import _native as N
    bound = {name for name, _, _ in N.SIGNATURES}
    assert set(declared_functions()) == bound


def test_struct_layout_matches_header(tmp_path):
    """ctypes mirrors of the ABI structs agree with the C compiler's layout of include/gwo.h."""
    import subprocess
    from flink_amd import _native as N
    structs = {"gwo_config": N.GwoConfig, "gwo_out": N.GwoOut, "gwo_side_out": N.GwoSideOut,
               "gwo_gen_spec": N.GwoGenSpec, "gwo_heap_state_ids": N.GwoHeapStateIds,
               "gwo_comm_waits": N.GwoCommWaits}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "gwo.h"', "int main(void){"]
    for cname, py in structs.items():
        lines.append(f'printf("{cname} __sizeof__ %zu\\n", sizeof({cname}));')
        for fname, _ in py._fields_:
            lines.append(f'printf("{cname} {fname} %zu\\n", offsetof({cname}, {fname}));')
    lines.append("return 0;}")
    c = tmp_path / "layout.c"
    c.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(c), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n")
    for line in filter(None, out):
        cname, field, val = line.split()
        py = structs[cname]
        want = ctypes.sizeof(py) if field == "__sizeof__" else getattr(py, field).offset
        assert int(val) == want, (cname, field)


def test_missing_library_fails_loudly(tmp_path):
    from flink_amd import _native as N
    with pytest.raises(N.NativeLibraryMissing):
        N.load(str(tmp_path / "libgwo.so"))


def test_status_strings():
    from flink_amd import _native as N
    lib = N.load()
    assert lib.gwo_status_string(0) == b"GWO_OK"
    assert lib.gwo_status_string(3) == b"GWO_ERR_KEY_GROUP"


def test_config_init_defaults():
    from flink_amd import _native as N
    lib = N.load()
    cfg = N.GwoConfig()
    lib.gwo_config_init(ctypes.byref(cfg))
    assert cfg.abi_version == N.GWO_ABI_VERSION and cfg.max_parallelism == 128 and cfg.key_group_end == 127


def test_python_assigner_validation():
    import flink_amd as F
    with pytest.raises(ValueError, match="abs\\(offset\\) < size"):
        F.TumblingEventTimeWindows.of(10, 20)
    with pytest.raises(ValueError, match="abs\\(offset\\) < slide"):
        F.SlidingEventTimeWindows.of(10, 5, 5)
    with pytest.raises(ValueError, match="0 < size"):
        F.EventTimeSessionWindows.withGap(0)
    r = F.compute_key_group_range_for_operator_index(32768, 8, 3)
    assert (r.start_key_group, r.end_key_group) == (12288, 16383)
