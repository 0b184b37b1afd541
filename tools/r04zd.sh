set -o pipefail
# the king-walk games test, then the whole GPU suite
OUT=gpurun_out/r04zd
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_games.py -x -q --timeout 120 --timeout-method thread -k king_walk > $OUT/king_walk.log 2>&1 || { tail -40 $OUT/king_walk.log; exit 1; }
tail -1 $OUT/king_walk.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
