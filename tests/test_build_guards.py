"""Build guards that need no GPU: the product build refuses the measurement-only RPT_EXP_* macros
(they make kernels skip work), the variant build still accepts them, and the test-only RCCL seam
(RPT_TESTING_HOOKS) is compiled only into the test build."""
import os
import subprocess

import pytest

from conftest import PKG, REPO

HIPCC = "/opt/rocm/bin/hipcc"
SRC = os.path.join(PKG, "csrc", "rpt_gpu.hip")


def preprocess(*defines):
    cmd = [HIPCC, "-E", "-std=c++17", "--offload-arch=gfx950", f"-I{REPO}/include", f"-I{PKG}/csrc", SRC, "-o", os.devnull]
    cmd += [f"-D{d}" for d in defines]
    return subprocess.run(cmd, capture_output=True, text=True)


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
@pytest.mark.parametrize("macro", ["RPT_EXP_PART_STOP=1", "RPT_EXP_SCATTER_SKIP=1", "RPT_EXP_STORE_SKIP_ZERO=1",
                                   "RPT_EXP_NO_PASS_WRITE=1"])
def test_product_build_refuses_measurement_macros(macro):
    r = preprocess("RPT_PRODUCT_BUILD=1", macro)
    assert r.returncode != 0 and "measurement macros are not allowed" in r.stderr
    assert preprocess(macro).returncode == 0  # tools/build_variants.sh (no RPT_PRODUCT_BUILD) may use them
    assert preprocess("RPT_PRODUCT_BUILD=1").returncode == 0


def test_product_makefile_defines_product_build():
    mk = open(os.path.join(PKG, "Makefile")).read()
    assert "PRODUCT := -DRPT_PRODUCT_BUILD=1" in mk and "$(HIPFLAGS) $(PRODUCT)" in mk
    assert "RPT_TESTING_HOOKS" not in mk.replace("# ", "")


def syntax_check(*defines):
    cmd = [HIPCC, "-fsyntax-only", "--cuda-host-only", "-std=c++17", f"-I{REPO}/include", f"-I{PKG}/csrc", SRC]
    cmd += [f"-D{d}" for d in defines]
    return subprocess.run(cmd, capture_output=True, text=True)


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
@pytest.mark.parametrize("macro", ["RPT_SLICE_UNROLL=2", "RPT_L1_TILE_ROWS=8192", "RPT_NT_REC_LOADS=1"])
def test_product_build_pins_tuning_macros(macro):
    """Tuning macros other than the defaults the GPU suite runs are for A/B variants only."""
    r = syntax_check("RPT_PRODUCT_BUILD=1", macro)
    assert r.returncode != 0 and "must keep their tested defaults" in r.stderr
    assert syntax_check(macro).returncode == 0
