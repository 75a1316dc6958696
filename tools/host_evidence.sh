#!/bin/bash
# Host-path evidence in one GPU call: the C++ mirror test, host_bench --create (CREATE_BF sink / flush / pinned
# cache sweep) and --chain (pipelined USE_BF chains), and the CPU restatement of the chains on the same host.
# Outputs under gpurun_out/host_evidence/.
set -e
cd "$(dirname "$0")/.."
out=gpurun_out/host_evidence
mkdir -p "$out"
timeout -k 10 240 ./tests/cpp/build/test_host_mirror > "$out/mirror.log" 2>&1
timeout -k 10 300 ./tools/host_bench/build/host_bench --create > "$out/create.jsonl" 2> "$out/create.err"
timeout -k 10 240 ./tools/host_bench/build/host_bench --chain > "$out/chain.jsonl" 2> "$out/chain.err"
timeout -k 10 400 bash tools/host_cpu_chain.sh > "$out/cpu_chain.jsonl" 2> "$out/cpu_chain.err"
echo done
