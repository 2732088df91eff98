#!/bin/bash
# relaxed first landing wait (_rw) vs production; fp8 long-K one-wave schedules
O=gpurun_out/r3s2_rw
mkdir -p $O
timeout -k 10 240 python -u tools/asm_lab.py --dtype bf16 --shapes 8192,4096x4096x16384,16384 --variants 136,180,140,181,150,182 --rounds 3 > $O/b.jsonl 2> $O/err &&
timeout -k 10 300 python -u tools/asm_lab.py --dtype fp8 --shapes 8192,4096,4096x4096x16384,16384x16384x1024 --variants 200,250,251,253,202,210,212,220,252 --rounds 3 > $O/f.jsonl 2>> $O/err
