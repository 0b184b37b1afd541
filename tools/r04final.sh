set -o pipefail
# round-4 profile at the round-4 final code: default bench line, kernel-trace stats, PMC passes (expand, big16m, small1m), plan/stream per-kernel passes
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/profile_round.sh r04z || exit 1
bash tools/pmc_kernels.sh r04z_kx expand || exit 1
