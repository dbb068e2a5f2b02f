#!/bin/bash
# Session: the GPU suite on the default library (zero records for culled splats).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
STEPS=tests bash tools/gpu_r05.sh
