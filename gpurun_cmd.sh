mkdir -p gpurun_out; export TMPDIR=/tmp
RPT_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 1 --probe-rows 2e8 > gpurun_out/bench_n2.log 2>&1; echo "n2 rc=$?"; grep '^{' gpurun_out/bench_n2.log | tail -c 1200
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -2
