set -o pipefail
# round-end rehearsal + profile with the column-sliced stream (GN_OPT_STREAM_SLICES 3 default)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/r04final_check.sh && bash tools/r04final.sh
