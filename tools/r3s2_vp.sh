#!/bin/bash
# VP DMA form and PA in the asm pipeline (K not a power of two)
O=gpurun_out/r3s2_vp
mkdir -p $O
timeout -k 10 300 python -u tools/asm_lab.py --dtype bf16 --shapes 8192,12288,8192x8192x12288,12288x12288x10240 --variants 136,190,191,193,150 --rounds 3 > $O/b.jsonl 2> $O/err &&
timeout -k 10 300 python -u tools/asm_lab.py --dtype fp8 --shapes 8192,12288,8192x8192x12288 --variants 200,260,261,262,263,220 --rounds 3 > $O/f.jsonl 2>> $O/err &&
timeout -k 10 200 python -u tools/gemm_sweep.py --variants p0,p48,p47 --shapes 12288,8192x8192x12288,12288x12288x10240 --rounds 2 > $O/prod_bf16.jsonl 2>> $O/err
