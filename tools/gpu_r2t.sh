# rows kernel in one 16-wave workgroup per CU (OPT bit 10) vs the product shapes, with priority
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2t
mkdir -p $O
for r in a b; do
EXPLORE_FILTER="nib G32 CH8 NBUF2 AUX2 wg/cu1 opt2 | 768 xw31:29,nib16w G32" timeout -k 10 300 ./tools/crc_explore 4096 $((1<<20)) 12 10 > $O/explore_4k_$r.log 2>&1
EXPLORE_FILTER="nib G16 CH4 NBUF2 AUX2 wg/cu2 opt2 | 256 xw31:29,nib16w G16" timeout -k 10 300 ./tools/crc_explore 1024 $((1<<22)) 12 10 > $O/explore_1k_$r.log 2>&1
EXPLORE_FILTER="crc G16 CH4 NBUF2 AUX2 wg/cu2 opt256 xw31:29,crc16w G16" timeout -k 10 300 ./tools/crc_explore 3072 $((1<<20)) 12 10 > $O/explore_3k_$r.log 2>&1
EXPLORE_FILTER="crc G64 CH4 NBUF2 AUX2 wg/cu1 opt256 xw31:29,crc16w G64" timeout -k 10 300 ./tools/crc_explore 65536 $((1<<16)) 12 10 > $O/explore_64k_$r.log 2>&1
done
echo ALLDONE
