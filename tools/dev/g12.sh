# dev (round 6): per-op k_attn_seq K/V ring depth 2 vs 3 (experiment builds libq3t_nb2 / nb3): 64-slot talker step on
# the launch-per-op graph (Q3T_PERSIST_TKB=0) at KV positions 266 and 500
set -o pipefail
cd $GRAFT_REPO_ROOT
for V in nb2 nb3 nb2 nb3; do
  echo "== $V"
  Q3T_DEV_LIB=$V Q3T_PERSIST_TKB=0 timeout -k 10 120 python3 tools/dev/stage_only.py 0 64 266 20 || exit 1
  Q3T_DEV_LIB=$V Q3T_PERSIST_TKB=0 timeout -k 10 120 python3 tools/dev/stage_only.py 0 64 500 20 564 || exit 1
done
