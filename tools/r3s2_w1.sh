#!/bin/bash
O=gpurun_out/r3s2_w1
mkdir -p $O
timeout -k 10 300 python -u tools/asm_lab.py --dtype fp8 --shapes 4096x4096x16384,4096x4096x32768,4096x8192x8192 --variants 200,210,202,212,220,260,261 --rounds 3 > $O/f.jsonl 2> $O/err &&
timeout -k 10 300 python -u tools/asm_lab.py --dtype bf16 --shapes 4096,12288,12288x12288x10240,16384 --variants 136,150,190,194,195 --rounds 3 > $O/b.jsonl 2>> $O/err
