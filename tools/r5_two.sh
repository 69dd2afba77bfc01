#!/bin/bash
# the two-chain 4 KiB plan: A/B against the product, then lib_timing of each library (LD_LIBRARY_PATH has no
# effect on lib_timing's rpath, so the variant is copied over a scratch copy of the tree's lib directory)
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${TAG:-r5x}; mkdir -p $O
timeout -k 10 300 python -u tools/ab_libs.py abbuild/r5fix/libpriskv_crc.so abbuild/r5two/libpriskv_crc.so --rounds=5 --streams=2 --cases=1Mix4KiB+65536x4KiB+4096x64KiB > $O/ab.jsonl 2> $O/ab.err || exit $?
