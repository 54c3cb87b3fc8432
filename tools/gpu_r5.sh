#!/bin/bash
# round-5 development runs (one GPU box): the load-shape microbenchmark, then
# the GPU tests named in $T (default: the golden-digest tests)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 ./tools/membench3 > gpurun_out/mb3.log 2>&1 && cat gpurun_out/mb3.log || exit 1
T=${T:-"tests/test_gpu_parity.py::test_pages_4k_golden_digests tests/test_gpu_parity.py::test_pages_8k_4088_4092_golden tests/test_gpu_parity.py::test_varlen_configs_exact_batches tests/test_xxh3.py::test_gpu_pages_golden tests/test_xxh3.py::test_gpu_varlen_configs_exact_batches"}
timeout -k 10 400 python -u -m pytest $T -x -v --timeout 120 --timeout-method thread > gpurun_out/t5.log 2>&1; rc=$?
tail -15 gpurun_out/t5.log; exit $rc
