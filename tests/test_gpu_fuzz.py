"""Seeded randomized parity sweep: random filter sizes, batch sizes, key types, NULL patterns,
dictionary vectors and row selections; every applicable probe strategy and insert strategy must give
the oracle's filter words and survivors. Bit-exact."""
import os

import numpy as np
import pytest
import torch

import golden_util as gu
import rpt_oracle as orc

pytestmark = pytest.mark.gpu

PROBE = {"gather": 1, "lds": 2, "partitioned": 3, "bucketed": 4}
INSERT = {"atomic": 1, "partitioned": 2, "bucketed": 3}


@pytest.fixture(scope="module")
def rpt():
    if not torch.cuda.is_available():
        pytest.fail("gpu test run without a visible GPU")
    import rpt_amd

    rpt_amd.load()
    torch.cuda.set_device(0)
    return rpt_amd


def dev(a):
    if a.dtype == np.uint64:
        a = a.view(np.int64)
    if a.dtype == np.uint32:
        a = a.view(np.int32)
    return torch.from_numpy(np.ascontiguousarray(a)).to("cuda:0")


def case(seed):
    rng = np.random.default_rng(seed)
    log_nb = int(rng.choice([4, 9, 13, 14, 15, 16, 17, 18, 21, 22, 23, 24]))  # 15-17: the hybrid LDS/L2 probe too
    dtype = np.int64 if rng.random() < 0.6 else np.int32
    n_build = int(rng.integers(1, 400_000))
    n_probe = int(rng.choice([1, 63, 511, 513, 16383, 16385, int(rng.integers(1, 700_000))]))
    info = np.iinfo(dtype)
    build = rng.integers(info.min, info.max, size=n_build, dtype=dtype, endpoint=True)
    hit = rng.random(n_probe) < rng.choice([0.0, 0.1, 0.9])
    probe = np.where(hit, build[rng.integers(0, n_build, n_probe)],
                     rng.integers(info.min, info.max, size=n_probe, dtype=dtype, endpoint=True)).astype(dtype)
    null_rate = float(rng.choice([0.0, 0.0, 0.05, 0.5]))
    b_valid = gu.validity_words(rng.random(n_build) >= null_rate) if null_rate else None
    p_valid = gu.validity_words(rng.random(n_probe) >= null_rate) if null_rate else None
    use_dict = rng.random() < 0.3
    use_rowsel = rng.random() < 0.3
    return dict(log_nb=log_nb, dtype=dtype, build=build, probe=probe, b_valid=b_valid, p_valid=p_valid,
                use_dict=use_dict, use_rowsel=use_rowsel, rng=rng)


# RPT_FUZZ_SEEDS seeds from RPT_FUZZ_SEED_BASE (tools/gpu_soak.sh sweeps more of them)
@pytest.mark.parametrize("seed", range(int(os.environ.get("RPT_FUZZ_SEED_BASE", "0")),
                                       int(os.environ.get("RPT_FUZZ_SEED_BASE", "0")) + int(os.environ.get("RPT_FUZZ_SEEDS", "24"))))
def test_random_configuration(rpt, seed):
    c = case(seed)
    lnb, rng = c["log_nb"], c["rng"]
    w = orc.new_words(lnb)
    orc.insert_keys(w, lnb, c["build"], validity=c["b_valid"])
    lib = rpt.load()
    for ins_name, ins in INSERT.items():
        if ins == 2 and not lib.rpt_probe_strategy_supported(3, lnb):
            continue
        if ins == 3 and not lib.rpt_probe_strategy_supported(4, lnb):
            continue
        bf = rpt.BloomFilter(log_num_blocks=lnb)
        bf.insert(dev(c["build"]), validity=dev(c["b_valid"]) if c["b_valid"] is not None else None, strategy=ins)
        assert np.array_equal(bf.export_words(), w), f"insert {ins_name}"
        # rebuild in place: the deferred clear is consumed by the insert (whole-slice stores) or settled
        # first (a reader in between, or an insert that cannot store whole slices)
        bf.clear()
        if rng.random() < 0.5:
            assert bf.lookup_sel(dev(c["probe"][:1000])).numel() == 0, f"{ins_name}: probe after clear"
        bf.insert(dev(c["build"]), validity=dev(c["b_valid"]) if c["b_valid"] is not None else None, strategy=ins)
        assert np.array_equal(bf.export_words(), w), f"rebuild {ins_name}"
    # probe: optionally through a dictionary and a row selection
    probe, key_sel, row_sel = c["probe"], None, None
    n = probe.size
    if c["use_dict"]:
        key_sel = rng.integers(0, probe.size, size=n).astype(np.uint32)
    if c["use_rowsel"]:
        row_sel = np.sort(rng.choice(n, size=max(1, n // 2), replace=False)).astype(np.uint32)
    rows = row_sel if row_sel is not None else np.arange(n, dtype=np.uint32)
    phys = key_sel[rows] if key_sel is not None else rows
    ref_local = orc.probe_keys(w, lnb, probe, key_sel=np.ascontiguousarray(phys.astype(np.uint32)),
                               validity=c["p_valid"])
    ref = rows[ref_local].astype(np.uint32)
    for name, st in PROBE.items():
        if not lib.rpt_probe_strategy_supported(st, lnb):
            continue
        bf.probe_strategy = st
        kw = dict(validity=dev(c["p_valid"]) if c["p_valid"] is not None else None,
                  key_sel=dev(key_sel) if key_sel is not None else None,
                  row_sel=dev(row_sel) if row_sel is not None else None)
        sel = bf.lookup_sel(dev(probe), **kw).cpu().numpy().view(np.uint32)
        assert np.array_equal(sel, ref), f"seed {seed} probe {name} log_nb {lnb}"
