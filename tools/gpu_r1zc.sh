set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r1zc
mkdir -p $O
timeout -k 10 200 python tools/ab_xcd.py 31:29 12 > $O/ab_3129.log 2>&1
timeout -k 10 200 python tools/ab_xcd.py 41:39 12 > $O/ab_4139.log 2>&1
timeout -k 10 200 python tools/ab_xcd.py 29:31 12 > $O/ab_2931.log 2>&1
timeout -k 10 200 python tools/ab_xcd.py 31:29 12 65536 > $O/ab_3129_64k.log 2>&1
echo ALLDONE
