mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 ./tests/cpp/build/test_host_mirror; echo "mirror rc=$?"
timeout -k 10 500 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
