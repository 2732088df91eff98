#!/bin/bash
# fused-epilogue (EPI=2) lab A/B: bf16 then fp8, knock-outs alongside (tools/asm_lab.py)
set -o pipefail
O=gpurun_out/r3s2_ef
mkdir -p $O
timeout -k 10 240 python -u tools/asm_lab.py --dtype bf16 --shapes 8192,16384,4096x4096x16384 --variants 136,170,171,172,173,160,161 --rounds 3 > $O/b.jsonl 2> $O/err &&
timeout -k 10 240 python -u tools/asm_lab.py --dtype fp8 --shapes 8192,16384,4096 --variants 200,240,241,242,243,230,231 --rounds 3 > $O/f.jsonl 2>> $O/err &&
timeout -k 10 300 python -u tools/asm_lab.py --dtype fp8 --shapes 16384x16384x4096,8192x8192x16384,16384x16384x1024,12288,16384x8192x8192 --variants 200,202,220,222,240,243 --rounds 2 > $O/sq.jsonl 2>> $O/err
