#!/bin/bash
# deferred C stores (EPI 7) vs production
O=gpurun_out/r3s2_ds
mkdir -p $O
timeout -k 10 240 python -u tools/asm_lab.py --dtype bf16 --shapes 8192,16384x16384x4096,8192x8192x2048 --variants 136,196,161 --rounds 4 > $O/b.jsonl 2> $O/err &&
timeout -k 10 240 python -u tools/asm_lab.py --dtype fp8 --shapes 8192,16384x16384x4096,8192x8192x2048 --variants 200,264,231 --rounds 4 > $O/f.jsonl 2>> $O/err
