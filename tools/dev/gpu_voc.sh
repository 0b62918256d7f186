#!/bin/bash
# dev: vocoder parity tests + FULL 512-frame timing (single and batched)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_vocoder.py tests/test_codebook_usage.py tests/test_quant.py tests/test_gpu_long.py -k "vocoder or codebook or quant" -x -v -s --timeout 300 --timeout-method thread -m gpu > gpurun_out/voc.log 2>&1
rc=$?
grep -E "PASS|FAIL|passed|failed|Error|max\|d\|" gpurun_out/voc.log | head -40
[ $rc -eq 0 ] || { tail -40 gpurun_out/voc.log; exit $rc; }
timeout -k 10 300 python3 tools/dev/voc_only.py 512 0 ${VOC_U:-16}
