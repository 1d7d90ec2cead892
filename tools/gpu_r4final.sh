#!/bin/bash
# Round-4 end measurement: kernel traces + HBM traffic passes of the three workloads (tools/pmc_all.sh), then the
# default bench line and the MFMA-busy passes (tools/final_pass.sh); every step time-limited, a failure ends the script
set -u
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
TAG=r4 bash tools/pmc_all.sh || exit $?
TAG=r4 bash tools/final_pass.sh || exit $?
echo r4final done
