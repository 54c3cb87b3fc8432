#!/bin/bash
# round 3: rocprofv3 kernel stats of zipf / chunks on the extent route vs the previous routes
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
CFGS="3:4096 1:4096" WORKLOADS=zipf bash tools/prof_routes.sh || exit 1
CFGS="3:4096 2:4096" WORKLOADS=chunks bash tools/prof_routes.sh || exit 1
