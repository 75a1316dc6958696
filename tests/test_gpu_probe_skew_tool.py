"""tools/probe_skew.py (the skewed-key timings behind DESIGN §5's skew table) with the oracle as its checker
(VERDICT r05 item 3): every run it times, at its full size of 2^27 rows with one hot key on 10 % / 100 % of them,
must return the oracle's survivors, and gather and partitioned must agree."""
import io
import json
import os
import sys

import numpy as np
import pytest
import torch

import rpt_oracle as orc
from conftest import REPO

pytestmark = pytest.mark.gpu


@pytest.mark.timeout(300)
def test_probe_skew_tool_runs_match_oracle():
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import probe_skew

    words = {}

    def check(keys, n_build, survivors):
        if n_build not in words:
            lnb = orc.log_num_blocks(n_build)
            w = orc.new_words(lnb)
            orc.build_mt(w, lnb, orc.synth_build_keys(n_build), max(1, min(16, len(os.sched_getaffinity(0)))))
            words[n_build] = (w, lnb)
        w, lnb = words[n_build]
        want = orc.probe_keys(w, lnb, keys.cpu().numpy()).astype(np.int64)
        assert np.array_equal(survivors, want)

    out = io.StringIO()
    probe_skew.run(check=check, builds=(10**7,), fractions=(0.1, 1.0), out=out)
    rows = [json.loads(x) for x in out.getvalue().splitlines()]
    assert len(rows) == 4 and len(words) == 1 and all(r["checked"] == "oracle" for r in rows), rows
    assert torch.cuda.is_available()
