"""dev: replay one captured stage graph (0 talker step, 1 CP frame) for PMC collection; prints mean ms."""
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(R, "qwen3-tts-jetson_amd"), os.path.join(R, "tests")]
import q3t  # noqa: E402
from q3t_testutil import synth_dir  # noqa: E402

stage, B, pos, iters = (int(a) for a in (sys.argv[1:5] + ["0", "1", "266", "10"][len(sys.argv) - 1:]))
max_ctx = int(sys.argv[5]) if len(sys.argv) > 5 else pos + 64
tts, _ = synth_dir("full")
eng = q3t.Engine(tts, None, max_slots=B, max_ctx=max_ctx)
print(f"stage {stage} B {B} pos {pos} ctx {max_ctx}: {eng.time_stage(stage, B, pos, iters):.4f} ms (replays {iters + 1})")
eng.close()
