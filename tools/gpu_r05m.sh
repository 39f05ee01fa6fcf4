#!/bin/bash
# round 5 box pass 13: full -m gpu suite with prop32 on by default (new tests/test_gpu_prop32.py first)
set -o pipefail
out=gpurun_out/r05m
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_prop32.py > $out/pytest_prop32.log 2>&1 || { tail -40 $out/pytest_prop32.log; exit 1; }
tail -3 $out/pytest_prop32.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $out/pytest_gpu.log 2>&1 || { tail -40 $out/pytest_gpu.log; exit 1; }
tail -3 $out/pytest_gpu.log
