#!/bin/bash
# round 6 session 5 (new container): smoke, the GPU suite and the default bench on the rebuilt tree,
# then the C5 (book2) rocprofv3 passes of the path-exact kernel as it stands (VERDICT r05 item 1's
# starting point)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r06
SKIP_PROF=1 bash tools/gpu_session.sh || exit $?
PROF_CFGS="c5:7:2048:2048:64" bash tools/prof_configs.sh || exit 3
