# one stream against batches alternating over 2 / 4 streams (tail overlap), 4 KiB / 64 KiB / 1 MiB
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4d
mkdir -p $O
for bs in 4096 65536 1048576; do
  timeout -k 10 200 python tools/two_stream_probe.py $bs >> $O/two_stream.jsonl 2>> $O/two_stream.err
done
echo ALLDONE
