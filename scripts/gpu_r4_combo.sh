#!/bin/bash
# One GPU session: scripts/gpu_r4_mixchol.sh, then an interleaved library A/B
# (scripts/lib_ab.sh) when LIBS is set.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
if [ "${SKIP_MIXCHOL:-0}" != 1 ]; then
  bash scripts/gpu_r4_mixchol.sh || exit $?
fi
if [ -n "$LIBS" ]; then
  RTAG=${ABTAG:-r4_ab} bash scripts/lib_ab.sh || exit $?
fi
