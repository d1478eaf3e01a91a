"""CPU: tools/amd-gpu-discovery.sh keeps the command-line and output contract of the reference's GPU
discovery script (GPUDriver.java:72-91 runs it with "<amount> <args>" and parses comma-separated
indices), against a fake KFD topology."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCRIPT = os.path.join(ROOT, "tools", "amd-gpu-discovery.sh")


@pytest.fixture
def topo(tmp_path):
    nodes = tmp_path / "nodes"
    for i, simds in enumerate([0, 1024, 1024, 1024]):   # node 0 = CPU, nodes 1..3 = GPUs
        d = nodes / str(i)
        d.mkdir(parents=True)
        (d / "properties").write_text(f"cpu_cores_count {0 if simds else 64}\nsimd_count {simds}\n")
    return tmp_path


def run(topo, *args, env_extra=None):
    env = dict(os.environ, GWO_KFD_TOPOLOGY=str(topo / "nodes"))
    env.pop("HIP_VISIBLE_DEVICES", None)
    env.update(env_extra or {})
    p = subprocess.run(["bash", SCRIPT, *map(str, args)], capture_output=True, text=True, env=env)
    return p.returncode, p.stdout.strip()


def test_non_coordination(topo):
    assert run(topo, 2) == (0, "0,1")
    assert run(topo, 3) == (0, "0,1,2")
    assert run(topo, 4)[0] == 1            # "Could not get enough GPU resources."
    assert run(topo, 0) == (0, "")
    assert run(topo, 2, env_extra={"HIP_VISIBLE_DEVICES": "2"})[0] == 1
    assert run(topo, 1, env_extra={"HIP_VISIBLE_DEVICES": "2"}) == (0, "0")


def test_coordination_mode(topo):
    f = topo / "coord"
    assert run(topo, 2, "--enable-coordination-mode", "--coordination-file", f) == (0, "0,1")
    held = sorted(line.split() for line in f.read_text().splitlines())
    assert [h[0] for h in held] == ["0", "1"] and all(h[1] == str(os.getpid()) for h in held)
    # devices 0 and 1 are held by a live process (this one): only device 2 is left
    assert run(topo, 2, "--enable-coordination-mode", "--coordination-file", f)[0] == 1
    assert run(topo, 1, "--enable-coordination-mode", "--coordination-file", f) == (0, "2")
    # an entry whose owner has exited is reclaimed
    f.write_text("0 999999999\n1 %d\n" % os.getpid())
    assert run(topo, 2, "--enable-coordination-mode", "--coordination-file", f) == (0, "0,2")


def test_bench_counts_gpus_without_hip(topo, monkeypatch):
    """bench.py's spawning parent counts GPUs from the same KFD topology (no HIP call before the ranks start)."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    for v in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(v, raising=False)
    assert bench.kfd_gpu_count(str(topo / "nodes")) == 3
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "1,2")
    assert bench.kfd_gpu_count(str(topo / "nodes")) == 2
    assert bench.kfd_gpu_count(str(topo / "missing")) == 0
