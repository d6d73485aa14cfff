#!/bin/bash
# r4j: head re-check after the container re-creation: GPU tests, smoke, the driver's bench line,
# the device-stamped timeline (synchronous frame + the 20-frame region)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_check.sh tests smoke bench_driver timeline
