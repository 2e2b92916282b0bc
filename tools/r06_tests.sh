#!/bin/bash
# Round-6 GPU check of selected tests (TESTS, pytest node ids / -k expression
# via PYARGS), one pytest process under its own time limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=${OUT:-gpurun_out/r06/tests}
mkdir -p $OUT
timeout -k 10 ${TLIM:-900} python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 300 --timeout-method thread $PYARGS \
  > $OUT/pytest.log 2>&1
rc=$?
tail -15 $OUT/pytest.log
exit $rc
