"""The driver's multi-GPU bench run, rehearsed end to end on ONE GPU.

`bench.py --gpus N` at N > 1 runs the headline (sharded C2 build, OR merge, merge check, sharded probe) and
then the `c5_merge` section: every rank inserts its shard of the N x rows build column into the 8 GiB filter
sized for 8e9 rows, the partials are OR-merged, the merged filter is checked against a single build of all
rows on every rank, and every rank probes its slice (the cross-GPU counterpart of PhysicalCreateBF::Combine,
reference src/operators/physical_create_bf.cpp:244-275). The driver's 8-GPU node runs it over RCCL; a
one-GPU box cannot (RCCL refuses two ranks on one device), so here the same script runs with
RPT_BENCH_BACKEND=gloo: N ranks share cuda:0, and every merge is the torch.distributed composition
(reported as torch_merge_ms, never as or_merge_ms). What this executes at N = 2, 4 and 8 (the driver's scaling
run makes N = 2, 4, 8) is everything of that run except the RCCL transport: the rank launch, the sharding, the merge check, the reductions over ranks,
the per-rank device-memory report and the record assembly.

bench.py starts its ranks itself (torch.distributed.run, before any GPU call in the ranks); this test starts
bench.py as a child process, whose output goes to gpurun_out/ so a long run shows progress.
"""
import json
import os
import subprocess
import sys
import time

import pytest

from conftest import REPO

pytestmark = pytest.mark.gpu

C5_FILTER_BYTES = 8 << 30
ROWS = 2 * 10**7


def run_bench(world: int, tmp_path):
    out_dir = os.path.join(REPO, "gpurun_out")
    os.makedirs(out_dir, exist_ok=True)
    log = os.path.join(out_dir, f"bench_rehearsal_n{world}.log")
    cmd = [sys.executable, "-u", os.path.join(REPO, "bench.py"), "--gpus", str(world), "--steps", "2", "--warmup", "1",
           "--probe-rows", "2e7", "--no-cpu-baseline", "--c5-rows-per-rank", str(ROWS), "--c5-merge-reps", "1"]
    env = dict(os.environ, RPT_BENCH_BACKEND="gloo")
    with open(log, "w") as f:
        p = subprocess.Popen(cmd, stdout=f, stderr=subprocess.STDOUT, env=env, cwd=REPO, start_new_session=True)
        try:
            rc = p.wait(timeout=840)
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, 9)
            p.wait()
            pytest.fail(f"bench.py --gpus {world} (gloo rehearsal) did not finish; see {log}")
    text = open(log).read()
    assert rc == 0, text[-4000:]
    lines = [x for x in text.splitlines() if x.startswith("{")]
    assert len(lines) == 1, text[-4000:]  # ONE JSON line, from rank 0
    return json.loads(lines[0])


@pytest.mark.timeout(900)
@pytest.mark.parametrize("world", [2, 4, 8])
def test_bench_multi_rank_rehearsal(world, tmp_path):
    t0 = time.monotonic()
    line = run_bench(world, tmp_path)
    # the headline: whole-node rate over N ranks, the C2 merge checked, no RCCL number reported
    assert line["n_gpus"] == world and line["scaling"] == "weak"
    assert line["value"] > 0 and line["config"]["probe_rows_per_gpu"] == 2 * 10**7
    assert line["build"]["merge_check"].startswith("bit-identical"), line["build"]
    assert line["build"]["or_merge_ms"] is None and line["build"]["torch_merge_ms"] > 0
    assert "cpu_baseline" not in line
    # ranks sharing one GPU: the stream calibration would time 8 concurrent streams, so it is skipped and says so
    assert line["stream_calibration"].startswith("skipped: ranks share one GPU"), line["stream_calibration"]
    assert line["roofline"]["stream_GBps"] is None
    # the C5 section at this N
    c5 = line["c5_merge"]
    assert c5["n_gpus"] == world and c5["rows_per_rank"] == ROWS and c5["build_rows"] == world * ROWS
    assert c5["filter_bytes"] == C5_FILTER_BYTES
    assert c5["merge_check"].startswith("bit-identical"), c5
    assert c5["or_merge_ms"] is None and c5["or_merge_ms_reps"] is None  # never an RCCL number from gloo
    assert c5["torch_merge_ms"] > 0 and len(c5["torch_merge_ms_reps"]) == 1
    assert "gloo rehearsal" in c5["merge_path"]
    assert c5["insert_ms"] > 0 and c5["probe_ms"] > 0
    assert 0.09 < c5["survivors_rank0"] / ROWS < 0.2  # p = 0.1 plus the filter's false positives
    mem = c5["device_memory"]
    assert mem["ranks_per_device"] == world
    assert len(mem["section_peak_bytes_per_rank"]) == world
    # each rank holds at least its filter and the merge check's reference filter at once
    assert all(p >= 2 * C5_FILTER_BYTES for p in mem["section_peak_bytes_per_rank"]), mem
    assert all(p <= mem["device_total_bytes"] for p in mem["device_peak_used_bytes_per_rank"]), mem
    assert set(mem["rank0_phase_used_bytes"]) == {"insert", "merge", "merge_timed", "merge_check", "probe"}
    # each rank's own footprint: at least its filter + the reference filter, and the 8 ranks' sum fits the device
    own = mem["rank_own_peak_bytes_per_rank"]
    assert len(own) == world and all(2 * C5_FILTER_BYTES <= p for p in own), own
    assert set(mem["rank0_own_phase_bytes"]) == {"insert", "merge", "merge_timed", "merge_check", "probe"}
    assert 0 < c5["wall_s"] < time.monotonic() - t0
