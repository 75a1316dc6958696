mkdir -p gpurun_out; export TMPDIR=/tmp
rm -rf gpurun_out/prof_c5
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5 -o c5 -- python3 bench.py --filter-rows 8e9 --build-rows 1e9 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_c5.log 2>&1 || { tail -5 gpurun_out/prof_c5.log; exit 1; }
head -30 gpurun_out/prof_c5/c5_kernel_stats.csv | cut -d, -f1-4 | cut -c1-150
