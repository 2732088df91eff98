#!/bin/bash
O=gpurun_out/r3s2_zc
mkdir -p $O
timeout -k 10 240 python -u tools/asm_lab.py --dtype bf16 --shapes 8192,16384,8192x8192x2048,4096x4096x16384 --variants 136,197,150,198 --rounds 4 > $O/b.jsonl 2> $O/err &&
timeout -k 10 240 python -u tools/asm_lab.py --dtype fp8 --shapes 8192,16384,8192x8192x2048,16384x16384x1024 --variants 200,265,220,266 --rounds 4 > $O/f.jsonl 2>> $O/err
