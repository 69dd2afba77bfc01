# per-wave finish times: read roof vs nibble-fold CRC, XCD weights on/off (explorer)
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1zze
mkdir -p $O
EXPLORE_FILTER="nib G32 CH8 NBUF2 AUX2 wg/cu1 opt2 xw31:29,rooft,nib G32 CH8 NBUF2 AUX2 wg/cu1 opt10,roof G32 CH8 NBUF2 AUX2 wg/cu1 xw" timeout -k 10 300 ./tools/crc_explore 4096 $((1<<20)) 8 50 > $O/explore_4k_wave_timing_roof.log 2>&1
echo ALLDONE
