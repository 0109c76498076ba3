#!/bin/bash
# round-6: statistics batch finished on the device (config 3's wall); the default bench line
export TMPDIR=/tmp
tools/gpu_run.sh \
  "r6/fin_tests:300:python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py" \
  "r6/fin_bench:600:python bench.py"
