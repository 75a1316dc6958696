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


def test_c5_merge_record_schema():
    """The `c5_merge` object bench.py adds at N > 1: merge time as the median of the
    timed reps, GB/s per GPU = 2 (W-1)/W S / t and per link = 2 S / W / t, the node-wide probe rate."""
    S = 8 << 30
    rec = bench.c5_merge_record(8, S, 10**9, 7.5, [0.30, 0.20, 0.25], 8.6, 12345, "bit-identical", 120000)
    for k in ("what", "n_gpus", "filter_bytes", "rows_per_rank", "build_rows", "insert_ms", "or_merge_ms",
              "or_merge_ms_reps", "or_merge_GBps_per_gpu", "or_merge_GBps_per_link", "probe_ms",
              "probe_keys_per_s_node", "survivors_rank0", "merge_check", "collective_timeout_ms"):
        assert k in rec, k
    assert rec["build_rows"] == 8 * 10**9 and rec["or_merge_ms"] == pytest.approx(250.0)
    assert rec["or_merge_GBps_per_gpu"] == pytest.approx(2 * 7 / 8 * S / 0.25 / 1e9)
    assert rec["or_merge_GBps_per_link"] == pytest.approx(2 / 8 * S / 0.25 / 1e9)
    assert rec["probe_keys_per_s_node"] == pytest.approx(8e9 / 8.6e-3)
    json.dumps(rec)
    one = bench.c5_merge_record(1, S, 10**7, 1.0, [0.001], 2.0, 1, "bit-identical", 1000)
    assert one["or_merge_GBps_per_gpu"] is None and one["or_merge_GBps_per_link"] is None  # no peer traffic
    # the torch composition (gloo rehearsal, --merge torch): torch_merge_ms only, never an or_merge number
    t = bench.c5_merge_record(2, S, 2 * 10**7, 1.0, [3.0], 2.0, 5, "bit-identical", None, native=False,
                              merge_path="torch (gloo rehearsal)", mem={"ranks_per_device": 2}, wall_s=40.0)
    assert t["torch_merge_ms"] == pytest.approx(3000.0) and t["torch_merge_ms_reps"] == [3000.0]
    for k in ("or_merge_ms", "or_merge_ms_reps", "or_merge_GBps_per_gpu", "or_merge_GBps_per_link"):
        assert t[k] is None, k
    assert t["device_memory"] == {"ranks_per_device": 2} and t["wall_s"] == 40.0
    assert rec["torch_merge_ms"] is None and "device_memory" not in rec
    json.dumps(t)


def test_c5_merge_flags(monkeypatch):
    assert bench.C5_FILTER_ROWS == 8 * 10**9 and bench.C5_ROWS_PER_RANK == 10**9
    monkeypatch.setattr(sys, "argv", ["bench.py"])
    a = bench.parse()
    assert not a.c5_merge and not a.no_c5_merge and a.c5_rows_per_rank == 1e9 and a.c5_merge_reps == 3
    assert a.collective_timeout_ms is None
    monkeypatch.setattr(sys, "argv", ["bench.py", "--c5-merge", "--c5-rows-per-rank", "1e7", "--collective-timeout-ms", "5000"])
    a = bench.parse()
    assert a.c5_merge and a.c5_rows_per_rank == 1e7 and a.collective_timeout_ms == 5000


def test_kernel_events_flag(monkeypatch):
    # per-kernel timing events run in a second pass by default (they cost ~25 us per step inside the timed steps)
    monkeypatch.setattr(sys, "argv", ["bench.py"])
    assert not bench.parse().kernel_events_in_timed_region
    monkeypatch.setattr(sys, "argv", ["bench.py", "--kernel-events-in-timed-region"])
    assert bench.parse().kernel_events_in_timed_region
