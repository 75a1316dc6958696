"""bench.py host logic (no GPU): rank launch contract, exact-instantiation PMC lookup, algorithmic
bytes per kernel, the CPU-baseline thread count."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402  (stdlib-only at import time)


def test_gpus_must_match_world_size():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=60)
    assert r.returncode != 0 and "--gpus 2 but WORLD_SIZE=1" in r.stderr


def test_launch_command_starts_n_ranks(monkeypatch):
    seen = {}

    def fake_call(cmd):
        seen["cmd"] = cmd
        return 7

    monkeypatch.setattr(bench.subprocess, "call", fake_call)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--config", "C5"])
    assert bench.launch_ranks(4) == 7
    cmd = seen["cmd"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"] and "--nproc-per-node=4" in cmd
    assert "127.0.0.1" in cmd and cmd[-4:] == ["--gpus", "4", "--config", "C5"]


def test_pmc_traffic_exact_instantiation(tmp_path, monkeypatch):
    d = tmp_path / "profiles" / "pmc"
    d.mkdir(parents=True)
    (d / "C3.json").write_text(json.dumps({"round": "t", "kernels": {
        "partition_kernel<0,true,false,2,0>": {"hbm_bytes_per_launch": 3.0},
        "slice_probe_kernel": {"avg_ms": 1.0}}}))
    monkeypatch.setattr(bench, "REPO", str(tmp_path))
    assert bench.pmc_traffic("partition_kernel<0,true,false,2,0>", "C3")["bytes_per_launch"] == 3.0
    # another instantiation, a bare name, a kernel without byte counters, another config: not profiled
    assert bench.pmc_traffic("partition_kernel<0,true,false,1,0>", "C3") is None
    assert bench.pmc_traffic("partition_kernel", "C3") is None
    assert bench.pmc_traffic("slice_probe_kernel", "C3") is None
    assert bench.pmc_traffic("partition_kernel<0,true,false,2,0>", "C2") is None


@pytest.mark.parametrize("name,expect", [
    ("partition_kernel<0,true,false,1,0>", 8 * 100), ("partition_kernel<1,true,false,1,0>", 8 * 100),
    ("partition_kernel<3,true,false,1,0>", 0), ("probe_bits_kernel<0,true,true,1024>", 8 * 100),
    ("bucket_scatter_kernel<0,true>", 8 * 100), ("unpermute_sel_kernel<1>", 4 * 7), ("compact_kernel", 4 * 7),
    ("slice_probe_kernel", 0), ("tile_count_kernel", 0), ("bucket_unpermute_kernel", 0)])
def test_algorithmic_bytes(name, expect):
    assert bench.algorithmic_bytes(name, 100, 7) == expect


def test_cpu_share():
    n = bench.cpu_share()
    assert 1 <= n <= len(os.sched_getaffinity(0))


def test_configs():
    assert bench.CONFIGS["C2"][0](1) == 10**7 and bench.CONFIGS["C3"][1](8) == 10**8
    assert bench.CONFIGS["C5"][0](8) == 8 * 10**9 and bench.CONFIGS["C5"][1](1) == 8 * 10**9
    assert bench.config_tag("C2", "i32") == "C2-i32"
