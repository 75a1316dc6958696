set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do for v in fresh pool sets; do
  timeout -k 10 300 abvar/$v/host_bench --host-path > gpurun_out/abhost_${v}_$rep.jsonl 2>&1 || { echo "$v failed"; tail -3 gpurun_out/abhost_${v}_$rep.jsonl; exit 1; }
  echo "$v $rep done"
done; done
