#!/bin/bash
# Full -m gpu suite on the box, one process, per-test timeout; log under gpurun_out/.
out=gpurun_out/${1:-tests}
mkdir -p $out
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread \
  ${@:2} > $out/pytest.log 2>&1
rc=$?
tail -30 $out/pytest.log
exit $rc
