# Split-K reduction knock-outs (tools-only lab cases 300-307, wrong results by design): where v57's
# reduction time goes. 300 = the production kernel built in the lab.
OUT=gpurun_out/${SK_OUT:-r6s15}; mkdir -p $OUT
timeout -k 10 400 python -u tools/asm_lab.py --shapes 2560x2560x8192,2048x4096x8192,2048x2048x16384 --variants 300,301,302,303,305,307 --rounds 3 > $OUT/splitk_ko.jsonl 2>&1
rc=$?; grep -v amdgpu.ids $OUT/splitk_ko.jsonl | grep -i "best\|summary" | head -20; exit $rc
