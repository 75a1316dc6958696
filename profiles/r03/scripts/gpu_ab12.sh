#!/usr/bin/env bash
# r03: the fused small probe loading all of a wave's segments before probing any (zero-copy keys: one PCIe
# round trip instead of one per segment): GPU parity tests, then host-bench per-vector / small-batch lines of
# HEAD's build ("base") and the working tree's.
set -o pipefail
mkdir -p gpurun_out/libbase
cp duckdb-robust-predicate-transfer_amd/build/variants/librpt_gpu_base.so gpurun_out/libbase/librpt_gpu.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_host_mirror.py tests/test_gpu_fuzz.py tests/test_readme_join.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_ab12.txt 2>&1 || { tail -30 gpurun_out/t_ab12.txt; exit 1; }
tail -1 gpurun_out/t_ab12.txt
for rep in 1 2; do
  LD_LIBRARY_PATH=$PWD/gpurun_out/libbase timeout -k 10 300 ./tools/host_bench/build/host_bench > gpurun_out/hb_base_$rep.jsonl 2>/dev/null || exit 1
  timeout -k 10 300 ./tools/host_bench/build/host_bench > gpurun_out/hb_pre_$rep.jsonl 2>/dev/null || exit 1
  for v in base pre; do echo "$v $rep"; grep -E "LookupSelBatch\", \"chunks_per_call\": (1|8|16), \"pipeline_rows\": -1|\"LookupSel\", \"threads\": (1|16)|UseBF::Execute\", \"filters\": (1|3)" gpurun_out/hb_${v}_$rep.jsonl | cut -c1-150; done
done
