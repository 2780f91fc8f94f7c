#!/bin/bash
# r02: GPU suite (receiver first), each step time-limited; stop at the first failure
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_receiver.py -x -v -s --timeout 120 --timeout-method thread > gpurun_out/pytest_rx.log 2>&1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_all.log 2>&1
