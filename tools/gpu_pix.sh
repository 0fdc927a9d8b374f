#!/bin/bash
# page-index GPU tests, then rocprof evidence for the given configs
cd "$(dirname "$0")/.."
tools/gpu_steps.sh "300 pix_tests python -u -m pytest tests/test_page_index.py -x -q --timeout 120 --timeout-method thread -rf" || exit $?
grep -q " passed" gpurun_out/pix_tests.log && ! grep -q "failed" gpurun_out/pix_tests.log || exit 1
[ -n "$EVIDENCE" ] && tools/evidence.sh $EVIDENCE
exit 0
