#!/bin/bash
O=gpurun_out/r3s2_rw2
mkdir -p $O
timeout -k 10 240 python -u tools/asm_lab.py --dtype bf16 --shapes 8192,8192x8192x4096,16384x16384x4096 --variants 136,180,150,182 --rounds 5 > $O/b.jsonl 2> $O/err &&
timeout -k 10 300 python -u tools/asm_lab.py --dtype fp8 --shapes 8192,16384,8192x8192x16384 --variants 200,250,253,210,220,252 --rounds 4 > $O/f.jsonl 2>> $O/err
