# in-call split: head on the caller stream, a back part forked onto a second stream to fill the head's tail
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4f
mkdir -p $O
for bs in 4096 65536 1048576; do
  timeout -k 10 200 python tools/split_tail_probe.py $bs >> $O/split_tail.jsonl 2>> $O/split_tail.err
done
echo ALLDONE
