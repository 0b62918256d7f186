#!/bin/bash
# dev: bit-for-bit A/B of the per-op batched talker (k_attn_seq) between two library variants (Q3T_DEV_LIB names)
set -o pipefail
A=$1; B=$2
Q3T_DEV_LIB=$A timeout -k 10 200 python3 -u tools/dev/attn_ab.py gpurun_out/attn_$A.npz || exit 1
Q3T_DEV_LIB=$B timeout -k 10 200 python3 -u tools/dev/attn_ab.py gpurun_out/attn_$B.npz || exit 1
python3 - "$A" "$B" <<'PY'
import sys
import numpy as np
a = np.load(f"gpurun_out/attn_{sys.argv[1]}.npz")
b = np.load(f"gpurun_out/attn_{sys.argv[2]}.npz")
print("hidden equal", np.array_equal(a["h"], b["h"]), "logits equal", np.array_equal(a["l"], b["l"]))
PY
