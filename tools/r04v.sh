set -o pipefail
# round-4 profile at commit 452d877: default bench line, kernel-trace stats, PMC passes (expand, big16m, small1m), plan/stream per-kernel passes
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/profile_round.sh r04v || exit 1
bash tools/pmc_kernels.sh r04v_kx expand || exit 1
