#!/bin/bash
# nontemporal C stores vs the staged and fused epilogues (tools/asm_lab.py)
O=gpurun_out/r3s2_nt
mkdir -p $O
timeout -k 10 240 python -u tools/asm_lab.py --dtype bf16 --shapes 8192,4096x4096x16384,16384 --variants 136,162,170,174,160 --rounds 3 > $O/b.jsonl 2> $O/err &&
timeout -k 10 240 python -u tools/asm_lab.py --dtype fp8 --shapes 8192,4096,16384x16384x1024 --variants 200,232,240,244,230 --rounds 3 > $O/f.jsonl 2>> $O/err
