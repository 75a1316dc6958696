"""Where a CREATE_BF's filter runs: rpt::PlanPushdown, the decision a DuckDB shim makes in
SetupDynamicFilterPushdown (forward USE_BF passthrough, /root/reference/src/optimizer/rpt_optimizer.cpp:1436-1440,
1493-1494) and PhysicalCreateBF's PushDynamicFilters (src/operators/physical_create_bf.cpp:282-350), for every
input combination, against the reference's logic restated here. CPU mode must equal the reference; GPU mode keeps
the BF probe in USE_BF (no BFTableFilter in the scan) and pushes the same cheap scan filters."""
import os
import subprocess

from conftest import REPO

CPP = os.path.join(REPO, "tests", "cpp")


def reference(ft, fwd, tgt, rows, bf_empty, mm):
    """(passthrough, always_false, push_bf, push_minmax) of the reference (CPU) path."""
    if not (fwd and tgt):
        return 0, 0, 0, 0  # nothing pushed, USE_BF probes
    if rows == 0:
        return 1, 1, 0, 0  # USE_BF passthrough (marked at planning), always-false only
    push_bf = ft in (0, 1) and not bf_empty
    push_mm = ft in (0, 2) and mm
    return 1, 0, int(push_bf), int(push_mm)


def test_pushdown_plan_every_combination():
    subprocess.run(["make", "-s", "-C", CPP], check=True)
    out = subprocess.run([os.path.join(CPP, "build", "test_pushdown_plan")], capture_output=True, text=True,
                         check=True).stdout.split()
    assert len(out) == 2 * 3 * 2 * 2 * 2 * 2 * 2
    for line in out:
        dev, ft, fwd, tgt, rows, bfe, mm, passthrough, af, pbf, pmm, in_use = (int(x) for x in line.split(","))
        ref = reference(ft, fwd, tgt, rows, bfe, mm)
        if dev == 0:  # cpu: the reference exactly; the BF is probed in USE_BF only when nothing was pushed
            assert (passthrough, af, pbf, pmm) == ref, line
            assert in_use == int(not (fwd and tgt)), line
        else:  # gpu: no BFTableFilter ever; USE_BF probes unless minmax_only drops the BF (as the reference)
            assert pbf == 0, line
            assert (af, pmm) == ref[1:2] + ref[3:4], line
            forward_pushed = fwd and tgt
            assert passthrough == int(forward_pushed and ft == 2), line
            assert in_use == int(not forward_pushed or ft != 2), line
