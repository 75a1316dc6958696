"""rpt_amd — host-side Python mirror of the predicate-transfer Bloom filter seam over librpt_gpu.so.

The product path is librpt_gpu.so (HIP kernels for gfx950 behind the C-ABI in include/rpt_gpu.h).
This package binds it with ctypes for tests, benches and the multi-GPU (torch.distributed/RCCL)
OR-merge; the C++ host mirror of the DuckDB operators lives in include/rpt_host.hpp.
"""
from ._lib import (  # noqa: F401
    LIB_PATH,
    RPT_INSERT_ATOMIC,
    RPT_INSERT_AUTO,
    RPT_INSERT_BUCKETED,
    RPT_INSERT_PARTITIONED,
    RPT_PROBE_AUTO,
    RPT_PROBE_BUCKETED,
    RPT_PROBE_GATHER,
    RPT_PROBE_LDS,
    RPT_PROBE_PARTITIONED,
    RPT_KEY_HASH,
    RPT_KEY_I32,
    RPT_KEY_I64,
    RptError,
    load,
)
from .bloom import (  # noqa: F401
    BloomFilter,
    ProbeWorkspace,
    hash_columns,
    hash_keys,
    log_num_blocks_for_rows,
    make_column,
    needs_resize,
    probe_chain,
    synth_build_keys,
    synth_probe_keys,
    validity_from_mask,
    words_or_slices,
)
