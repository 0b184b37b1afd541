set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/profile_round.sh r04h || exit 1
bash tools/pmc_kernels.sh r04h_k small1m || exit 1
bash tools/pmc_kernels.sh r04h_kx expand || exit 1
