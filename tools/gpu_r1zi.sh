set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1zi
mkdir -p $O
F="opt2 xw,opt10 xw,roof G32 CH8 NBUF2 AUX2 wg/cu1 xw0"
EXPLORE_FILTER="$F" timeout -k 10 300 ./tools/crc_explore 4096 $((1<<20)) 8 20 > $O/explore_4k.log 2>&1
F="G64 CH4 NBUF2 AUX2 wg/cu1 opt0 xw,G64 CH4 NBUF2 AUX2 wg/cu1 opt8 xw,roof G64 CH4 NBUF2 AUX2 wg/cu2 xw0"
EXPLORE_FILTER="$F" timeout -k 10 300 ./tools/crc_explore 65536 65536 8 20 > $O/explore_64k.log 2>&1
for i in slice8 clmul vclmul; do PRISKV_CRC_HOST_IMPL=$i timeout -k 10 60 ./tools/host_key_bench priskv_amd/lib/libpriskv_crc.so >> $O/host_keys.jsonl; done
timeout -k 10 60 ./tools/host_key_bench oracle/_ref/libpriskv_ref_crc_O2.so >> $O/host_keys.jsonl
echo ALLDONE
