#!/bin/bash
# One GPU session: the -m gpu suite, then optional bench commands, each under its own time limit.
# A test FAILURE (rc 1) does not stop the session; a fault / abort / timeout (any other non-zero
# rc) does: nothing more runs on the GPU in this call.
#   bash tools/gpu_session.sh <tag> [pytest-args...]    (BENCH_CMDS: extra ';;'-separated commands)
tag=${1:?tag}; shift
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p $out
cd $GRAFT_REPO_ROOT
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest tests -m gpu -x -v --timeout 300 \
    --timeout-method thread "$@" > $out/gputest.log 2>&1
  rc=$?
  echo "pytest rc=$rc"; tail -3 $out/gputest.log
  ok $rc || exit $rc
fi
i=0
IFS=';;' read -ra CMDS <<< "${BENCH_CMDS:-}"
for c in "${CMDS[@]}"; do
  [ -z "$c" ] && continue
  i=$((i+1))
  echo "== cmd $i: $c"
  bash -c "$c" > $out/cmd$i.log 2> $out/cmd$i.err
  rc=$?
  echo "cmd $i rc=$rc"; tail -2 $out/cmd$i.log | cut -c1-600; tail -3 $out/cmd$i.err
  [ $rc -eq 0 ] || exit $rc
done
