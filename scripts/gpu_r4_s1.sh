#!/bin/bash
# Round-4 session 1: the store-layout micro-benchmark, then the mix_chol session
# (scripts/gpu_r4_mixchol.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r4_ubench
echo "== write_layout $(date +%T)"
timeout -k 10 120 scripts/ubench/write_layout > gpurun_out/r4_ubench/write_layout.txt 2>&1 || exit $?
cat gpurun_out/r4_ubench/write_layout.txt
bash scripts/gpu_r4_mixchol.sh
