"""A JOB-shaped predicate transfer through the C++ operators: the closest stand-in for BASELINE
config 4 (JOB-113 on job.duckdb, absent from the image) that runs here.

Four tables of INTEGER join keys with NULLs, already reduced by their base predicates, in JOB's shape:
    mi(movie_id, info_type_id)   fact, largest (the root under the largest_root heuristic)
    it(id)                       a dimension after its predicate (12 of 113 info types)
    t(id)                        title after its predicate (40 % of the ids)
    mc(movie_id)                 a second fact table hanging off title
    joins: mi.info_type_id = it.id, mi.movie_id = t.id, t.id = mc.movie_id
tests/cpp/test_job_transfer runs the forward + backward CREATE_BF / USE_BF schedule that GenerateStageModifications
emits for this tree (/root/reference/src/optimizer/rpt_optimizer.cpp:828-995) through rpt::CreateBF (parallel sink,
Combine, Finalize with its resize rule, the parallel source re-emitting the materialized rows into the next stage)
and rpt::UseBF (per-chunk Execute and the pipelined ExecuteBatch chain) on cuda:0. This test replays the same
schedule with the oracle (tests never trust the program's own bookkeeping):
  * every CREATE_BF's filter words == the oracle's filter over exactly the rows that reached it, sized by the same
    estimate and resize rule (physical_create_bf.cpp:352-419);
  * every USE_BF's survivors == the oracle's AND of its filters over exactly its input rows
    (physical_use_bf.cpp:112-197);
  * the join of the reduced tables == the join of the unreduced tables (the result a query sees must not change:
    test_job_queries.sh:256 diffs query outputs with and without the extension). DuckDB is absent: the join is
    numpy's, NULL keys never match.
"""
import os
import subprocess

import numpy as np
import pytest

import rpt_oracle as orc
from conftest import REPO

CPP = os.path.join(REPO, "tests", "cpp")
BIN = os.path.join(CPP, "build", "test_job_transfer")


def pack(valid: np.ndarray) -> np.ndarray:
    """bool rows -> DuckDB ValidityMask words."""
    b = np.packbits(valid.astype(np.uint8), bitorder="little")
    b = np.concatenate([b, np.zeros((-b.size) % 8 + 8, dtype=np.uint8)])
    return b.view(np.uint64)


def make_tables(seed: int = 6):
    rng = np.random.default_rng(seed)
    n_title = 1_000_000
    t_id = np.sort(rng.choice(n_title, size=400_000, replace=False)).astype(np.int32)  # title after its predicate
    rng.shuffle(t_id)
    tables = {
        "t": {"id": (t_id, np.ones(t_id.size, bool))},
        "it": {"id": (rng.choice(113, size=12, replace=False).astype(np.int32), np.ones(12, bool))},
    }
    n_mi, n_mc = 1_500_000, 800_000
    tables["mi"] = {
        "movie_id": (rng.integers(0, n_title, n_mi).astype(np.int32), rng.random(n_mi) >= 0.01),
        "info_type_id": (rng.integers(0, 113, n_mi).astype(np.int32), rng.random(n_mi) >= 0.01),
    }
    tables["mc"] = {"movie_id": (rng.integers(0, int(n_title * 1.2), n_mc).astype(np.int32), rng.random(n_mc) >= 0.02)}
    # three of the selected info types never occur in mi: the backward pass must drop them from it
    it_ids = tables["it"]["id"][0]
    ity = tables["mi"]["info_type_id"][0]
    ity[np.isin(ity, it_ids[:3])] = it_ids[3]
    # one title id appears in NULL rows of mi too (a NULL row's key bytes are ignored: it never matches)
    mi_keys, mi_valid = tables["mi"]["movie_id"]
    mi_keys[~mi_valid] = t_id[0]
    est = {"f_mc": n_mc, "f_it": 113, "f_t": 1000, "f_mi": n_mi // 20, "f_t2": t_id.size}
    return tables, est


def write_inputs(d, tables, est):
    for tname, cols in tables.items():
        for cname, (keys, valid) in cols.items():
            keys.astype(np.int32).tofile(os.path.join(d, f"{tname}_{cname}.i32"))
            valid.astype(np.uint8).tofile(os.path.join(d, f"{tname}_{cname}.valid"))
    with open(os.path.join(d, "est.txt"), "w") as f:
        for k, v in est.items():
            f.write(f"{k} {v}\n")


def oracle_filter(keys, valid, est_rows):
    """CREATE_BF over these rows: sized for the estimate (uint32, physical_create_bf.cpp:187), resized at Finalize
    when the allocation gives < 8 bits per actual row (rpt_bf_needs_resize_alloc's rule)."""
    lnb = orc.log_num_blocks(est_rows & 0xFFFFFFFF)
    resized = keys.size > 0 and orc.needs_resize_alloc(lnb, keys.size)
    if resized:
        lnb = orc.log_num_blocks(keys.size)
    w = orc.new_words(lnb)
    if keys.size:
        orc.insert_keys(w, lnb, keys, validity=pack(valid))
    return w, lnb, resized


def oracle_use(filters, cols, rows):
    """USE_BF: the rows (table row ids) passing every filter (AND), each on its own key column."""
    keep = np.ones(rows.size, bool)
    for (w, lnb), (keys, valid) in zip(filters, cols):
        k, v = keys[rows], valid[rows]
        sel = orc.probe_keys(w, lnb, k, validity=pack(v))
        m = np.zeros(rows.size, bool)
        m[sel] = True
        keep &= m
    return rows[keep]


def np_join(lk, lrows, rk, rrows):
    """Equi-join of (lk, lrows) and (rk, rrows) (NULL rows already dropped): matching (lrow, rrow) pairs."""
    order = np.argsort(rk, kind="stable")
    rs = rk[order]
    lo = np.searchsorted(rs, lk, "left")
    hi = np.searchsorted(rs, lk, "right")
    cnt = hi - lo
    li = np.repeat(np.arange(lk.size), cnt)
    off = np.arange(cnt.sum()) - np.repeat(np.cumsum(cnt) - cnt, cnt)
    ri = order[np.repeat(lo, cnt) + off]
    return lrows[li], rrows[ri]


def join4(tables, rows):
    """mi ⋈ it ⋈ t ⋈ mc over the given row sets: sorted (mi, it, t, mc) row-id tuples."""
    def col(tn, cn):
        k, v = tables[tn][cn]
        r = rows[tn][v[rows[tn]]]  # NULL keys never join
        return k[r], r
    k1, r1 = col("mi", "info_type_id")
    k2, r2 = col("it", "id")
    mi_a, it_a = np_join(k1, r1, k2, r2)
    mi_keys, mi_valid = tables["mi"]["movie_id"]
    ok = mi_valid[mi_a]
    mi_a, it_a = mi_a[ok], it_a[ok]
    kt, rt = col("t", "id")
    pos_l, t_b = np_join(mi_keys[mi_a], np.arange(mi_a.size), kt, rt)
    mi_b, it_b = mi_a[pos_l], it_a[pos_l]
    km, rm = col("mc", "movie_id")
    t_keys = tables["t"]["id"][0]
    pos_l2, mc_c = np_join(t_keys[t_b], np.arange(t_b.size), km, rm)
    out = np.stack([mi_b[pos_l2], it_b[pos_l2], t_b[pos_l2], mc_c], axis=1)
    return out[np.lexsort(out.T[::-1])]


def read(d, name, dtype):
    return np.fromfile(os.path.join(d, name), dtype=dtype)


def test_job_transfer_schedule_oracle_only():
    """The schedule replayed by the oracle alone (no GPU): the reduced join equals the unreduced one and every
    table shrinks, so the GPU test below checks a transfer that removes rows without changing the result."""
    tables, est = make_tables()
    full = {tn: np.arange(next(iter(c.values()))[0].size) for tn, c in tables.items()}
    red = oracle_schedule(tables, est, full)
    assert all(red[f"final_{tn}"].size < full[tn].size for tn in ("mi", "it", "t", "mc"))
    want = join4(tables, full)
    got = join4(tables, {tn: np.sort(red[f"final_{tn}"]) for tn in full})
    assert want.shape[0] > 1000 and np.array_equal(got, want)


def oracle_schedule(tables, est, full, check=None):
    """The forward + backward schedule of tests/cpp/test_job_transfer.cpp over the oracle. `check(name, kind, value)`
    is called with every filter ("bf", (words, lnb, resized)) and every USE_BF's survivors ("use", row ids)."""
    check = check or (lambda *a: None)
    out = {}

    def create(name, tn, cn, rows):
        k, v = tables[tn][cn]
        w, lnb, resized = oracle_filter(k[rows], v[rows], est["f_mi" if name.startswith("f_mi") else name])
        check(name, "bf", (w, lnb, resized, rows.size))
        return w, lnb

    def use(name, filters, tn, cns, rows):
        r = oracle_use(filters, [tables[tn][c] for c in cns], rows)
        check(name, "use", r)
        return r

    f_mc = create("f_mc", "mc", "movie_id", full["mc"])
    f_it = create("f_it", "it", "id", full["it"])
    t_fwd = use("t_fwd", [f_mc], "t", ["id"], full["t"])
    f_t = create("f_t", "t", "id", t_fwd)
    mi_fwd = use("mi_fwd", [f_it, f_t], "mi", ["info_type_id", "movie_id"], full["mi"])
    f_mi_it = create("f_mi_it", "mi", "info_type_id", mi_fwd)
    f_mi_t = create("f_mi_t", "mi", "movie_id", mi_fwd)
    it_bwd = use("it_bwd", [f_mi_it], "it", ["id"], full["it"])
    t_bwd = use("t_bwd", [f_mi_t], "t", ["id"], t_fwd)
    f_t2 = create("f_t2", "t", "id", t_bwd)
    mc_bwd = use("mc_bwd", [f_t2], "mc", ["movie_id"], full["mc"])
    out.update(final_mi=mi_fwd, final_it=it_bwd, final_t=t_bwd, final_mc=mc_bwd)
    return out


def test_job_transfer_program_builds():
    subprocess.run(["make", "-s", "-C", CPP], check=True)
    out = subprocess.run(["ldd", BIN], capture_output=True, text=True, check=True).stdout
    assert "librpt_gpu.so" in out and "not found" not in out and "librpt_oracle" not in out


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_job_transfer_through_the_operators(tmp_path):
    subprocess.run(["make", "-s", "-C", CPP], check=True)
    tables, est = make_tables()
    d = str(tmp_path)
    write_inputs(d, tables, est)
    r = subprocess.run([BIN, d], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and "ALL OK" in r.stdout, r.stdout + r.stderr
    full = {tn: np.arange(next(iter(c.values()))[0].size) for tn, c in tables.items()}
    checked = []

    def check(name, kind, value):
        if kind == "bf":
            w, lnb, resized, rows = value
            lg, rs, n = (int(x) for x in open(os.path.join(d, f"bf_{name}.txt")).read().split())
            assert (lg, bool(rs), n) == (lnb, resized, rows), f"{name}: geometry / resize / rows"
            assert np.array_equal(read(d, f"bf_{name}.u64", np.uint64), w), f"{name}: filter words differ from the oracle"
        else:
            got = read(d, f"use_{name}.i64", np.int64)
            assert np.array_equal(np.sort(got), np.sort(value)), f"{name}: survivors differ from the oracle"
        checked.append(name)

    red = oracle_schedule(tables, est, full, check)
    assert len(checked) == 11
    for tn in ("mi", "it", "t", "mc"):  # what each join input holds after the transfer (the source's re-emission)
        got = read(d, f"final_{tn}.i64", np.int64)
        assert np.array_equal(np.sort(got), np.sort(red[f"final_{tn}"])), tn
        assert got.size < full[tn].size
    want = join4(tables, full)
    got = join4(tables, {tn: np.sort(read(d, f"final_{tn}.i64", np.int64)) for tn in full})
    assert want.shape[0] > 1000 and np.array_equal(got, want)
    # the estimate of 1000 for t's forward filter is under its 400k-row input: Finalize resized it
    assert open(os.path.join(d, "bf_f_t.txt")).read().split()[1] == "1"
