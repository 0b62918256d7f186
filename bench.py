#!/usr/bin/env python3
"""bench.py — frames/s + RTF of the MI355X Qwen3-TTS decode path (BASELINE.json metric, configs[1]).

A "step" = one utterance batch through the whole hot path: text projection + prefill, `--frames` audio frames
(talker step -> CB0 selection -> 16-pass code predictor -> step embedding, one hipGraph per frame) and the
vocoder over the produced codes.  Inputs (prompt ids) are tiny; weights and all state live in HBM.
Synthetic 0.6B-shaped weights (tools/q3t_synth.c, seed 0x51E3775), synthetic 16-token prompt, reference
sampling defaults (temperature 0.9, top-k 50, repetition penalty 1.05) with EOS masked for exactly --frames
frames (force_frames).

N GPUs: one process per GPU (torchrun), utterances sharded across ranks (weak scaling), barrier + max-over-ranks
timing.  Rank 0 prints ONE JSON line.  Multi-GPU start-up: local rank 0 reads the GGUF files, every
other rank parses only their headers and receives the packed weight blobs by RCCL broadcast over xGMI; barriers and
the max-over-ranks of the timer are RCCL all-reduces on the same communicator.  The 128-byte RCCL unique id travels
through a node-local file (single-node contract); no framework runtime is loaded beside libq3t.so.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "qwen3-tts-jetson_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))

SAMPLES_PER_FRAME = 1920           # 24 kHz / 12.5 Hz (src/trt_vocoder.h:50)
FRAME_SEC = 0.08
TALKER_WEIGHT_BYTES = 887_095_296  # 28 x 15,728,640 x 2 + 3072 x 1024 x 2
KV_BYTES_PER_POS = 114_688         # 28 layers x 2 (K,V) x 8 heads x 128 x 2 B
CP_PASS_BYTES = 5 * 15_728_640 * 2
CP_HEAD_BYTES = 2048 * 1024 * 2
HBM_PEAK_GBS = 8000.0              # MI355X_MICROARCH.md chip table (spec)
MFMA_PEAK_TFLOPS = 2500.0          # dense f16/bf16 MFMA, MI355X_MICROARCH.md (spec; sparsity figures excluded)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def _time_oracle(tts, tok, prompt, frames, vocoder_mode, threads, n, cfg0_frames):
    """one thread count: (a) prefill + n frames + the vocoder of those n frames, extrapolated to `frames`;
    (b) BASELINE configs[0] measured directly: one cfg0_frames-frame utterance end to end (prefill, frames, vocoder)"""
    import numpy as np
    from oracle_py import Oracle
    o = Oracle(tts, tok, threads=threads)
    spk = np.zeros(o.cfg["hidden"], np.float32)
    kw = dict(spk=spk, temperature=0.9, top_k=50, seed=1, rep=1.05)
    o.generate(prompt, max_len=1, force_frames=1, **kw)   # page the weights in (mmap) before anything is timed
    t0 = time.perf_counter()
    o.generate(prompt, max_len=1, force_frames=1, **kw)
    t1 = time.perf_counter()
    codes = o.generate(prompt, max_len=1 + n, force_frames=1 + n, **kw)
    t2 = time.perf_counter()
    t_frame = ((t2 - t1) - (t1 - t0)) / n
    t_prefill = max(0.0, (t1 - t0) - t_frame)
    t_voc = 0.0
    if vocoder_mode is not None:
        o.vocoder(codes[:8], vocoder_mode)   # vocoder weights paged in
        t3 = time.perf_counter()
        o.vocoder(codes, vocoder_mode)
        t_voc = (time.perf_counter() - t3) / len(codes)
    t4 = time.perf_counter()
    c0 = o.generate(prompt, max_len=cfg0_frames, force_frames=cfg0_frames, **kw)
    if vocoder_mode is not None:
        o.vocoder(c0, vocoder_mode)
    t_cfg0 = time.perf_counter() - t4
    o.close()
    total = t_prefill + frames * (t_frame + t_voc)
    return dict(total=total, t_prefill=t_prefill, t_frame=t_frame, t_voc=t_voc, n=len(codes), t_cfg0=t_cfg0,
                wall=time.perf_counter() - t0)


def cpu_baseline(tts, tok, prompt, frames, vocoder_mode, gpu):
    """The oracle (C restatement of the reference GGML-CPU path) timed on a bounded sample and extrapolated to the
    workload: t = t_prefill + frames * (t_frame + t_vocoder_per_frame), plus BASELINE configs[0] (one 32-frame utterance)
    measured end to end without extrapolation.  The vocoder convs run as ggml runs them (im2col rows of the f16-rounded
    input times the f16 kernel, f32 accumulation) on a register-blocked AVX2/F16C GEMM.  Main number at 4 threads: the
    reference never plumbs n_threads (src/qwen3_tts.h:32), so the ggml CPU backend runs its default
    GGML_DEFAULT_N_THREADS = 4 [ggml-upstream]; the all-cores figure (OMP_NUM_THREADS) is reported beside it.
    gpu: the GPU's own per-frame decode / vocoder times and configs[0] RTF, for the per-stage ratios."""
    res = {}
    allc = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    cfg0 = 32
    # samples sized to ~10-30 s of CPU work in total
    for threads, n in ((4, 64), (allc, 96)):
        r = _time_oracle(tts, tok, prompt, frames, vocoder_mode, threads, n, cfg0)
        rtf0 = r["t_cfg0"] / (cfg0 * FRAME_SEC)
        res[threads] = dict(
            value=round(frames / r["total"], 3), rtf=round(r["total"] / (frames * FRAME_SEC), 4),
            decode_only={"cpu_ms_per_frame": round(r["t_frame"] * 1e3, 2),
                         "gpu_ms_per_frame": round(gpu["decode_ms_per_frame"], 3),
                         "ratio": round(r["t_frame"] * 1e3 / gpu["decode_ms_per_frame"], 1)},
            vocoder_only=None if vocoder_mode is None else {
                "cpu_ms_per_frame": round(r["t_voc"] * 1e3, 2), "gpu_ms_per_frame": round(gpu["vocoder_ms_per_frame"], 4),
                "ratio": round(r["t_voc"] * 1e3 / gpu["vocoder_ms_per_frame"], 1)},
            configs0={"frames": cfg0, "cpu_s": round(r["t_cfg0"], 3), "cpu_rtf": round(rtf0, 4),
                      "gpu_rtf": round(gpu["cfg0_rtf"], 5), "rtf_ratio": round(rtf0 / gpu["cfg0_rtf"], 1)},
            sample=f"prefill + {r['n']} frames + vocoder of {r['n']} frames, then one {cfg0}-frame utterance end to "
                   f"end ({r['wall']:.1f} s of CPU work): t_prefill {r['t_prefill']:.2f}s, {r['t_frame'] * 1e3:.1f} "
                   f"ms/frame, vocoder {r['t_voc'] * 1e3:.1f} ms/frame, extrapolated to {frames} frames (the CPU's "
                   f"per-frame attention grows with the KV position: a {r['n']}-frame sample undercounts it at positions "
                   f"up to {frames + len(prompt)}, so the extrapolated CPU time, and the GPU/CPU ratio, are conservative)")
    r4 = res[4]
    return {"value": r4["value"], "unit": "frames/s", "cores": 4, "kind": "port", "rtf": r4["rtf"],
            "decode_only": r4["decode_only"], "vocoder_only": r4["vocoder_only"], "configs0": r4["configs0"],
            "sample": "oracle/q3t_oracle.c (GGML-CPU restatement, f16 weights, f16-rounded matmul inputs) on the full "
                      "0.6B synthetic model at the reference's ggml default of 4 threads: " + r4["sample"],
            "all_cores": {"cores": allc, **res[allc]}}


# ------------------------------------------------------------------------------------------ multi-process plumbing
class LocalCtrl:
    """world 1: nothing to synchronise across processes."""
    def barrier(self):
        pass

    def max(self, v):
        return v


class RcclCtrl:
    """barrier / max-over-ranks as RCCL all-reduces on the shared context's communicator."""
    def __init__(self, eng):
        self.eng = eng

    def barrier(self):
        self.eng.allreduce_max([0.0])

    def max(self, v):
        return float(self.eng.allreduce_max([v])[0])


def timed_steps(ctrl, sync, step, steps):
    """The contract's timed region: device fence + barrier, K steps, device fence + barrier, max over ranks."""
    sync()
    ctrl.barrier()
    t0 = time.perf_counter()
    for k in range(steps):
        step(k)
    sync()
    ctrl.barrier()
    return ctrl.max(time.perf_counter() - t0)


def _uid_path():
    # one file per torchrun job: every rank of a job shares MASTER_PORT and the launching agent (parent pid)
    return os.path.join(os.environ.get("Q3T_UID_DIR", "/tmp"),
                        f"q3t_rccl_uid_{os.environ.get('MASTER_PORT', '0')}_{os.getppid()}")


def exchange_uid(rank, make_uid, timeout=300.0):
    """rank 0 publishes the RCCL unique id (atomic rename); the other ranks poll for it."""
    path = _uid_path()
    if rank == 0:
        uid = make_uid()
        tmp = path + ".tmp"
        with open(tmp, "wb") as f:
            f.write(uid)
        os.replace(tmp, path)
        return uid
    t0 = time.time()
    while not os.path.exists(path):
        if time.time() - t0 > timeout:
            raise RuntimeError(f"rank {rank}: no RCCL id from rank 0 at {path} after {timeout:.0f} s")
        time.sleep(0.05)
    with open(path, "rb") as f:
        return f.read()


def release_uid():
    try:
        os.remove(_uid_path())
    except OSError:
        pass


def pmc_traffic(slots):
    """HBM bytes per talker-step replay from the newest committed rocprofv3 FETCH_SIZE pass
    (profiles/rNN_pmc_fetch_talker_step[_b64].txt, tools/dev/gpu.sh fetch; x2 gfx950 correction applied there)."""
    import glob
    import re
    suffix = "" if slots == 1 else f"_b{slots}"
    files = sorted(glob.glob(os.path.join(REPO, "profiles", f"r*_pmc_fetch_talker_step{suffix}.txt")))
    if not files:
        return None, None
    m = re.search(r"->\s*([0-9.]+) MB per replay", open(files[-1]).read())
    return (round(float(m.group(1)) * 1e6), os.path.relpath(files[-1], REPO)) if m else (None, None)


def pmc_file(tag):
    """newest committed MFMA-utilisation table (tools/dev/gpu.sh mfma: kernel trace + SQ_INSTS_MFMA / FETCH / WRITE)"""
    import glob
    files = sorted(glob.glob(os.path.join(REPO, "profiles", f"r*_pmc_mfma_{tag}.txt")))
    return os.path.relpath(files[-1], REPO) if files else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--frames", type=int, default=512)
    ap.add_argument("--batch", type=int, default=1, help="utterances per GPU")
    ap.add_argument("--vocoder", choices=["full", "chunk40", "none"], default="full")
    ap.add_argument("--cpu-baseline", choices=["on", "off"], default="on")
    ap.add_argument("--cfg", default="full", choices=["full", "tiny"])
    ap.add_argument("--roofline-pos", type=int, default=10 + 512 // 2,
                    help="KV position of the talker-step roofline measurement (mid-utterance of configs[1])")
    ap.add_argument("--stage-iters", type=int, default=20, help="graph replays timed for the roofline")
    ap.add_argument("--batched", type=int, default=64,
                    help="secondary measurement: this many concurrent utterances per GPU (BASELINE configs[2] at N=1, "
                         "configs[3] at N>1: weak scaling, value over all ranks); 0 = off")
    ap.add_argument("--serve", type=int, default=2048,
                    help="serving measurement (N=1): this many utterances with natural EOS (prompt lengths 10..120 "
                         "tokens) through --serve-slots slots, lock-step batches vs continuous batching; 0 = off")
    ap.add_argument("--serve-slots", type=int, default=256,
                    help="slots of the serving measurement (one context: the batched path is latency-bound at 64 "
                         "slots, 288 GB of HBM holds the KV of 256)")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import numpy as np
    import q3t
    from q3t_testutil import prompt as make_prompt, synth_dir

    voc_mode = {"full": q3t.VOCODER_FULL, "chunk40": q3t.VOCODER_CHUNK40, "none": None}[args.vocoder]
    max_ctx = max(args.frames, args.roofline_pos) + 32
    batched = args.batched
    serve_slots = args.serve_slots if args.serve > 0 and world == 1 else 0
    slots = max(args.batch, batched, serve_slots)
    weights = "local GGUF read"
    if world > 1:
        # rank 0 writes the synthetic GGUFs (node-local), then publishes the RCCL id; the others wait for it
        if rank == 0:
            tts, tok = synth_dir(args.cfg)
        uid = exchange_uid(rank, q3t.comm_unique_id if rank == 0 else None)
        if rank != 0:
            tts, tok = synth_dir(args.cfg)
        eng = q3t.Engine.shared(tts, tok if voc_mode is not None else None, local_rank, slots, max_ctx,
                                rank, world, uid)
        if rank == 0:
            release_uid()
        weights = f"rank 0 GGUF read + RCCL broadcast to {world - 1} rank(s)"
        ctrl = RcclCtrl(eng)
    else:
        tts, tok = synth_dir(args.cfg)
        eng = q3t.Engine(tts, tok if voc_mode is not None else None, device=0, max_slots=slots, max_ctx=max_ctx)
        ctrl = LocalCtrl()
    B = args.batch
    prompt = make_prompt(args.cfg)
    H = eng.cfg["hidden"]
    prompts = [prompt] * B
    spks = [np.zeros(H, np.float32)] * B
    stats = {"prefill_ms": 0.0, "frames_ms": 0.0, "vocoder_ms": 0.0}

    def step(k, prompts=prompts, spks=spks):
        codes = eng.generate(prompts, speakers=spks, max_len=args.frames, temperature=0.9, top_k=50,
                             repetition_penalty=1.05, seed=1000 * rank + k, force_frames=args.frames)
        pm, fm = eng.last_timing()
        stats["prefill_ms"] += pm
        stats["frames_ms"] += fm
        if voc_mode is not None:
            t = time.perf_counter()
            if len(codes) == 1:
                eng.vocoder(codes[0], voc_mode)
            else:   # utterance batches through shared launches (q3t_vocoder_decode_batch)
                eng.vocoder_batch(codes, voc_mode)
            stats["vocoder_ms"] += (time.perf_counter() - t) * 1e3
        return codes

    for w in range(args.warmup):
        step(-1 - w)
    for k in stats:
        stats[k] = 0.0
    elapsed = timed_steps(ctrl, eng.synchronize, step, args.steps)
    main_stats = dict(stats)
    ms_per_step = elapsed / args.steps * 1e3
    total_frames = world * B * args.frames * args.steps
    value = total_frames / elapsed

    # ---- per-stage GPU times for the CPU-baseline ratios: decode loop and vocoder per frame of the timed steps, and
    # BASELINE configs[0] (one 32-frame utterance, prefill + frames + vocoder) end to end, median of 5 wall-clock runs
    gpu_stage = {"decode_ms_per_frame": main_stats["frames_ms"] / (args.steps * args.frames),
                 "vocoder_ms_per_frame": main_stats["vocoder_ms"] / (args.steps * args.frames * B)}
    if rank == 0 and args.cpu_baseline == "on" and world == 1:
        t_c0 = []
        for k in range(6):
            eng.synchronize()
            t = time.perf_counter()
            c0 = eng.generate([prompt], speakers=[spks[0]], max_len=32, temperature=0.9, top_k=50,
                              repetition_penalty=1.05, seed=77, force_frames=32)
            if voc_mode is not None:
                eng.vocoder(c0[0], voc_mode)
            eng.synchronize()
            t_c0.append(time.perf_counter() - t)
        gpu_stage["cfg0_rtf"] = sorted(t_c0[1:])[2] / (32 * FRAME_SEC)

    pk = eng.persist_kernels()
    tk_kernel = ("k_tk_roles, persist_tk.hip: role-specialised workgroups, 2 per CU" if pk & 1 else
                 "k_persist<0,64>, persist.hip" if pk & 2 else "launch-per-op graph")
    cp_kernel = ("k_cp_roles, persist_cp.hip: role-specialised workgroups" if pk & 4 else
                 "k_persist<1,16>, persist.hip" if pk & 8 else "launch-per-op graph")

    # ---- roofline of the talker decode step (SURVEY §8(d) definition) at the mid-utterance position
    p_mid = args.roofline_pos
    t_talker = eng.time_stage(0, B, p_mid, args.stage_iters)
    talker_bytes = TALKER_WEIGHT_BYTES + KV_BYTES_PER_POS * (p_mid + 2) * B
    achieved = talker_bytes / (t_talker * 1e-3) / 1e9
    t_cp = eng.time_stage(1, B, p_mid, max(1, args.stage_iters // 2))
    cp_bytes = 16 * CP_PASS_BYTES + 15 * CP_HEAD_BYTES

    # ---- vocoder (MFMA-bound): algorithmic FLOPs of the loaded conv / projection shapes over the
    # measured vocoder time of the step; SQ_INSTS_MFMA evidence per kernel in profiles/rNN_pmc_mfma_vocoder.txt
    voc_flops = eng.vocoder_flops(args.frames) if voc_mode == q3t.VOCODER_FULL else None
    eng_voc_batch = 4096   # q3t_vocoder_set_batch_frames default

    def voc_roofline(voc_ms, n_utt, steps):
        if not voc_flops or voc_ms <= 0:
            return None
        tf = voc_flops * n_utt * steps / (voc_ms * 1e-3) / 1e12
        return {"bound": "mfma", "kernel": ("FULL vocoder of one utterance per call" if n_utt == 1 else
                                            f"FULL vocoder, {n_utt} utterances in batches of {eng_voc_batch} frames") +
                                           " (k_conv_mt implicit-GEMM convs on v_mfma_f32_32x32x16_f16, transposed convs "
                                           "one launch per conv)",
                "achieved": round(tf, 1), "peak": MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": round(tf / MFMA_PEAK_TFLOPS, 4), "flops_per_decode": round(voc_flops),
                "ms_per_decode": round(voc_ms / (n_utt * steps), 3), "mfma_pmc": pmc_file("vocoder")}

    # ---- secondary: BASELINE configs[2], `batched` concurrent utterances through the matrix-core path
    bres = None
    if batched > 0:
        bp = [prompt] * batched
        bs = [np.zeros(H, np.float32)] * batched
        for k in stats:
            stats[k] = 0.0
        step(-100, bp, bs)   # warm-up (graph capture for this slot count)
        for k in stats:
            stats[k] = 0.0
        b_steps = 3
        b_el = timed_steps(ctrl, eng.synchronize, lambda k: step(100 + k, bp, bs), b_steps) / b_steps
        bt = eng.time_stage(0, batched, p_mid, max(2, args.stage_iters // 4))
        bc = eng.time_stage(1, batched, p_mid, 2)
        b_bytes = TALKER_WEIGHT_BYTES + KV_BYTES_PER_POS * (p_mid + 2) * batched
        bres = {"config": (f"configs[2]: {batched} concurrent utterances x {args.frames} frames on one GPU"
                           if world == 1 else f"configs[3]: {world} x {batched} utterances x {args.frames} frames, "
                           f"utterance-sharded over {world} GPUs") +
                          f", vocoder({args.vocoder}) in utterance batches, temp 0.9 top-k 50",
                "value": round(world * batched * args.frames / b_el, 1), "unit": "frames/s",
                "ms_per_step": round(b_el * 1e3, 1), "n_gpus": world, "scaling": "weak",
                "x_realtime": round(args.frames * FRAME_SEC * batched * world / b_el, 1),
                "steps": b_steps, "breakdown_ms_per_step": {k: round(v / b_steps, 1) for k, v in stats.items()},
                "talker_step_ms": round(bt, 4), "cp_frame_ms": round(bc, 4),
                "roofline": {"bound": "hbm", "kernel": f"talker decode step at KV position {p_mid}, {batched} slots " + (
                                 "(ONE persistent launch, k_tkb, persist_tkb.hip: 28 layers + codec head + CB0 selection; "
                                 "MFMA tile jobs with LDS-DMA weights, granule / flag hand-offs, attention one workgroup "
                                 "per (slot, kv head) streaming the whole context)" if pk & 32 else
                                 "(MFMA f16 GEMMs on hoisted norms, split-K slabs, k_attn_seq: one workgroup per (slot, kv "
                                 "head) streaming the whole context: 7 launches per layer)"),
                             "achieved": round(b_bytes / (bt * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                             "frac": round(b_bytes / (bt * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                             "traffic": pmc_traffic(batched)[0], "traffic_source": pmc_traffic(batched)[1],
                             "bytes_per_launch": b_bytes, "launch_ms": round(bt, 4)},
                "cp_kernel": ("16-pass code-predictor frame of every slot, ONE persistent launch (k_cpb, persist_cpb.hip)"
                              if pk & 16 else "16-pass code-predictor frame, launch-per-op graph (decoder_stack_mm)"),
                "vocoder_roofline": voc_roofline(stats["vocoder_ms"], batched, b_steps),
                "mfma_pmc": pmc_file("talker_b64"), "mfma_pmc_cp": pmc_file("cp_b64")}

    # ---- serving: utterances of different lengths, lock-step batches (every batch runs until its
    # longest utterance ends) vs continuous batching (a finished slot is refilled between frames); codes only
    sres = None
    if args.serve > 0 and serve_slots > 0 and world == 1:
        rng = np.random.default_rng(2024)
        sp_prompts = []
        for i in range(args.serve):
            n = int(rng.integers(10, 121))
            sp_prompts.append(prompt[:4] + [(prompt[4 + j % (len(prompt) - 4)] + 13 * i + 7 * j) % 900 + 20
                                            for j in range(n - 4)])
        sp_spk = [np.zeros(H, np.float32)] * args.serve
        kw = dict(max_len=args.frames, temperature=0.9, top_k=50, repetition_penalty=1.05, seed=4242)
        eng.generate_queue(sp_prompts[:2 * serve_slots], speakers=sp_spk[:2 * serve_slots], max_active=serve_slots,
                           **dict(kw, max_len=2))   # warm-up: every slot's single-slot prefill graph
        eng.generate(sp_prompts[:serve_slots], speakers=sp_spk[:serve_slots], **dict(kw, max_len=2))
        eng.synchronize()
        t0 = time.perf_counter()
        lock = []
        for b0 in range(0, args.serve, serve_slots):
            lock += eng.generate(sp_prompts[b0:b0 + serve_slots], speakers=sp_spk[b0:b0 + serve_slots], **kw)
        eng.synchronize()
        t_lock = time.perf_counter() - t0
        t0 = time.perf_counter()
        queue = eng.generate_queue(sp_prompts, speakers=sp_spk, max_active=serve_slots, **kw)
        eng.synchronize()
        t_queue = time.perf_counter() - t0
        f_lock, f_queue = sum(len(c) for c in lock), sum(len(c) for c in queue)
        sres = {"config": f"{args.serve} utterances (prompts of 10..120 tokens, natural EOS, max {args.frames} frames) "
                          f"through {serve_slots} slots of one context, codes only (no vocoder), temp 0.9 top-k 50",
                "lockstep": {"frames": f_lock, "s": round(t_lock, 3), "value": round(f_lock / t_lock, 1),
                             "unit": "frames/s"},
                "continuous": {"frames": f_queue, "s": round(t_queue, 3), "value": round(f_queue / t_queue, 1),
                               "unit": "frames/s"},
                "lengths": {"min": min(len(c) for c in queue), "mean": round(f_queue / args.serve, 1),
                            "max": max(len(c) for c in queue)}}

    if rank == 0:
        res = {
            "metric": "audio frames/sec (12 Hz frames) + RTF, Qwen3-TTS-0.6B batch=1 and batch=8xN",
            "value": round(value, 2), "unit": "frames/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 2), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f16",
            "data": "synthetic (random-init 0.6B-shaped weights from tools/q3t_synth.c, 16-token prompt)",
            "config": {"workload": f"configs[1]: Qwen3-TTS-0.6B {B} utterance(s)/GPU x {args.frames} frames, "
                                   f"talker+code-predictor+vocoder({args.vocoder}) HIP path, temp 0.9 top-k 50",
                       "utterances_per_gpu": B, "frames": args.frames, "vocoder": args.vocoder,
                       "parallelism": f"utterance-sharded dp{world}", "weights": weights},
            "rtf": round(ms_per_step / 1e3 / (args.frames * FRAME_SEC), 5),
            "x_realtime": round(args.frames * FRAME_SEC * B / (ms_per_step / 1e3), 1),
            "breakdown_ms_per_step": {k: round(v / args.steps, 2) for k, v in main_stats.items()},
            "talker_step_ms": round(t_talker, 4), "cp_frame_ms": round(t_cp, 4),
            "roofline": {"bound": "hbm", "kernel": f"talker decode step at KV position {p_mid} (28 layers + codec head + "
                                                  "CB0 selection: ONE persistent launch, " + tk_kernel + ")"
                                                  if B == 1 else f"talker decode step at KV position {p_mid}, {B} slots",
                         "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": pmc_traffic(B)[0],
                         "traffic_source": pmc_traffic(B)[1],
                         "bytes_per_launch": talker_bytes, "launch_ms": round(t_talker, 4)},
            "vocoder_roofline": voc_roofline(main_stats["vocoder_ms"], B, args.steps),
            "cp_roofline": {"kernel": f"16-pass code-predictor frame, ONE persistent launch ({cp_kernel})",
                            "achieved": round(cp_bytes / (t_cp * 1e-3) / 1e9, 1), "unit": "GB/s",
                            "bytes_per_frame": cp_bytes, "note": "157 MB of CP weights re-read 16x per frame "
                            "(Infinity-Cache resident), algorithmic bytes / time"},
        }
        res["batched"] = bres
        res["serving"] = sres
        vr = res["vocoder_roofline"]
        res["mfma_frac"] = vr["frac"] if vr else None   # the MFMA-bound kernel's fraction (vocoder convs, §8(d))
        if args.cpu_baseline == "on" and world == 1:
            try:
                res["cpu_baseline"] = cpu_baseline(tts, tok if voc_mode is not None else None, prompt, args.frames,
                                                   voc_mode, gpu_stage)
            except Exception as e:  # the GPU number stands on its own
                res["cpu_baseline"] = {"value": None, "error": str(e)}
        else:
            res["cpu_baseline"] = None
        print(json.dumps(res), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
