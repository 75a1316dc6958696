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


def test_small_probe_rows_cover_every_segment():
    """RPT_SMALL_PROBE_ROWS (include/rpt_gpu.h) that is not a multiple of 16 waves x 512 rows
    would leave segments unprobed (their rows silently dropped); more than 64 segments overflow the one-wave
    sel-tail scan. The kernels static_assert both; the header's value obeys them."""
    import re

    hdr = open(os.path.join(REPO, "include", "rpt_gpu.h")).read()
    rows = int(re.search(r"#define RPT_SMALL_PROBE_ROWS (\d+)", hdr).group(1))
    assert rows % (512 * 16) == 0 and rows // 512 <= 64
    src = open(os.path.join(PKG, "csrc", "kernels", "probe_direct.hpp")).read()
    assert "static_assert(kSmallRows % (kSegRows * (kSmallThreads / 64)) == 0 && kSmallRows / kSegRows <= 64" in src


def test_product_library_reads_no_tuning_environment():
    """the product library's level-1 geometry and partition tile size ignore the tuning
    environment variables (only the variant builds of tools/build_variants.sh read them)."""
    lib = os.path.join(PKG, "build", "librpt_gpu.so")
    if not os.path.exists(lib):
        pytest.skip("product library not built")
    blob = open(lib, "rb").read()
    for var in (b"RPT_L1_GROUPS_MIN_ROWS", b"RPT_TILE_MULT_SLICES"):
        assert var not in blob, var
