set -o pipefail
# L1 probe: stream time and L2 hit rate of the planned expansion with L1 = 1024 vs 3072
OUT=gpurun_out/r04zg
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/l1_probe.py 1024 > $OUT/t1024.log 2>&1 || { tail -20 $OUT/t1024.log; exit 1; }
timeout -k 10 300 python -u tools/l1_probe.py 3072 > $OUT/t3072.log 2>&1 || { tail -20 $OUT/t3072.log; exit 1; }
grep l1 $OUT/t1024.log $OUT/t3072.log
timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $OUT/pmc_l2_1024 -o run -- python3 tools/l1_probe.py 1024 > $OUT/pmc1024.log 2>&1 || { tail -20 $OUT/pmc1024.log; exit 1; }
python tools/pmc_kernels_summary.py r04zg stream_eval > $OUT/sum.txt 2>&1; grep -i "hit\|==" $OUT/sum.txt
