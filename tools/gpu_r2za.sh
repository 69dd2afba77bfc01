# sub-KiB kernel: 16-wave workgroups with / without progress priority
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2za
mkdir -p $O
for bs in 32 64 256 512; do
timeout -k 10 120 ./tools/crc_explore $bs $(( (1<<32) / bs )) 10 > $O/small_$bs.log 2>&1
done
echo ALLDONE
