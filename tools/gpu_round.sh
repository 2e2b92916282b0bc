#!/bin/bash
# Round GPU call: parity tests + bench (tools/gpu_check.sh), then the round
# profile (tools/gpu_profile_round.sh); large per-dispatch traces are removed
# afterwards so gpurun_out/ stays under the copy-back limit.
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_check.sh; rc=$?
if [ $rc -eq 0 ]; then
  bash tools/gpu_profile_round.sh > gpurun_out/profile_round.log 2>&1; rc=$?
  echo "profile rc=$rc"; tail -5 gpurun_out/profile_round.log
fi
find gpurun_out -type f -size +1M ! -name "*stats*" -delete
du -sh gpurun_out
exit $rc
