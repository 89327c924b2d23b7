#!/usr/bin/env python3
"""Freeze-Omni MI355X benchmark: streaming speech-to-speech turns for N users per GPU.

metric (BASELINE.json): real-time factor + p50 first-audio-chunk latency, Qwen2-7B, N users/GPU.

One "step" = one full dialogue turn for every user on every rank (SURVEY.md §8(d) config 3 per GPU):
  listen : 10 s of synthetic 16 kHz PCM per user streamed in 160 ms chunks (framing A, 63 chunks);
           each chunk = fbank -> speech encoder -> adapter -> Qwen2-7B chunk prefill (per-user paged KV
           forked from a shared system prompt) -> dialog-state head (host read each chunk, as the reference)
  speak  : dialog_ss -> assistant-prefix prefill + 8 text tokens (benchmark policy: one sentence of 8
           tokens) -> AR speech decoder (EOS masked until 400 codec tokens = 10 s of 24 kHz audio) ->
           TiCodec vocoder per 40(+10+10) tokens -> silence-cut emission.
value = seconds of 24 kHz speech emitted by all users on all ranks / max-over-ranks wall seconds
(aggregate real-time factor, higher is better).  Also reported: per-user RTF (audio / (dialog_ss ->
last PCM)), p50/p90 first-audio latency (dialog_ss -> PCM of the first vocoder chunk known on the host,
the reference's "first PCM chunk" of assets/latency.png) and p50_first_emit_gated_ms (dialog_ss -> first
segment released by the find_min_sum_index silence gate; random-weight codec output has no 100 ms
quiet window, so the gate holds the audio until the final flush).
Weights: counter-hash synthetic weights at Qwen2-7B / paper geometry (configs/real), generated on
device; no checkpoint is on the box.  Launch for N>1 with torch.distributed.run (one rank per GPU).
"""
import argparse
import json
import math
import os
import sys
import time


def _blas_threads_from_argv(default=16):
    """--cpu-threads, read before numpy is imported so the BLAS pool is created at that size."""
    n = default
    for i, a in enumerate(sys.argv):
        if a == "--cpu-threads" and i + 1 < len(sys.argv):
            n = int(sys.argv[i + 1])
        elif a.startswith("--cpu-threads="):
            n = int(a.split("=", 1)[1])
    return n


for _k in ("OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS", "MKL_NUM_THREADS", "BLIS_NUM_THREADS"):
    os.environ[_k] = str(_blas_threads_from_argv())

import numpy as np  # noqa: E402

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "freeze-omni_amd"))


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--users", type=int, default=8, help="concurrent users per GPU")
    ap.add_argument("--config", default="real", choices=["real", "tiny"])
    ap.add_argument("--input-sec", type=float, default=10.0)
    ap.add_argument("--text-tokens", type=int, default=8)
    ap.add_argument("--codec-tokens", type=int, default=400)
    ap.add_argument("--top-k", type=int, default=1, help="speech decoder top_k (1 = parity/greedy)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pipeline", dest="pipeline", action="store_false",
                    help="listen chunk by chunk (default: encoder stage of chunk c+1 overlaps the LLM of chunk c)")
    ap.add_argument("--scenario", default="turn", choices=["turn", "duplex"],
                    help="turn: config 3 (default, the headline line); duplex: config 5 sessions")
    ap.add_argument("--duplex-sec", type=float, default=60.0, help="duplex: seconds of audio per session")
    ap.add_argument("--cpu-threads", type=int, default=16,
                    help="BLAS threads of the cpu_baseline leg (set before numpy is imported)")
    ap.add_argument("--no-single-user", action="store_true", help="skip the config-2 (1 user) leg")
    ap.add_argument("--out", default=None, help="also write the JSON line to this file")
    return ap.parse_args()


def synth_pcm(n, seed):
    """band-limited noise x 4 Hz syllabic AM at -20 dBFS, int16-quantised."""
    rng = np.random.default_rng(seed)
    t = np.arange(n) / 16000.0
    w = np.convolve(rng.standard_normal(n + 64), np.hanning(33), mode="same")[:n]
    w = w / (np.abs(w).max() + 1e-9)
    x = 0.1 * w * 0.5 * (1 + np.sin(2 * np.pi * 4 * t))
    return (np.round(x * 32767) / 32768.0).astype(np.float32)


class Turn:
    """Per-user state of one dialogue turn."""

    def __init__(self, engine, base_kv, pcm):
        from fo.speech import Framer
        self.kv = base_kv.fork()
        self.framer = Framer("A")
        self.pcm = pcm
        self.enc_cache = self.ada_cache = None
        self.pe = 0


def run_turn(engine, base_kv, pcms, args, sync):
    import torch
    from fo.speak import speak
    B = len(pcms)
    t_begin = time.perf_counter()
    turns = [Turn(engine, base_kv, p) for p in pcms]
    fb = engine.fbank("A")
    CH = turns[0].framer.chunk
    n_chunks = int(math.ceil(len(pcms[0]) / CH))
    pipe = engine.listen_pipe() if args.pipeline else None
    from fo import ops
    side = ops.engine_stream(engine.device, side=True)
    for c in range(n_chunks):
        wins, firsts = [], []
        for t in turns:
            seg = t.pcm[c * CH:(c + 1) * CH]
            if len(seg) < CH:
                seg = np.pad(seg, (0, CH - len(seg)))
            w, f = t.framer.push(seg)
            wins.append(w)
            firsts.append(f)
        if pipe is not None and c > 0:
            with torch.cuda.stream(side):   # the encoder stage's stream: no legacy-stream barrier
                feats = fb(np.stack(wins), firsts)
        else:
            feats = fb(np.stack(wins), firsts)
        items = [dict(identity="user", status="ipu_sl" if c == 0 else "ipu_cl", feats=feats[b], kv=t.kv,
                      enc_cache=t.enc_cache, ada_cache=t.ada_cache, pe_index=t.pe) for b, t in enumerate(turns)]
        if pipe is not None and c > 0:
            # steady state: this chunk's encoder stage overlaps the previous chunk's LLM stage
            pe_next, _ = pipe.push(items)
            for t, pe in zip(turns, pe_next):
                t.pe = pe
        else:
            for t, r in zip(turns, engine.listen(items)):
                t.enc_cache, t.ada_cache, t.pe = r["enc_cache"], r["ada_cache"], r["pe_index"]
    if pipe is not None:
        pipe.flush()
    # ---- dialog_ss (benchmark policy forces it at end of input, as bin/inference.py:138 does)
    sync()
    t_ss = time.perf_counter()
    eod = engine.tokenizer.eod_id
    pre = engine.prefix_ids["system"]
    text_ids = [[] for _ in turns]
    hiddens = []
    nxt, hid = engine.text_step([(t.kv, pre) for t in turns])
    for _ in range(args.text_tokens):
        hiddens.append(hid)
        for b in range(B):
            text_ids[b].append(nxt[b] if nxt[b] != eod else 0)
        if len(hiddens) == args.text_tokens:
            break
        nxt, hid = engine.text_step([(t.kv, [text_ids[b][-1]]) for b, t in enumerate(turns)])
    t_text = time.perf_counter()   # the last text step's ids were read back: the text stage is done
    D = engine.llm.D
    idim = engine.cfg["decoder_json"][0]
    items = []
    ids_d = torch.tensor(text_ids, dtype=torch.int32).to(engine.device)
    emb = engine.llm.embed(ids_d.view(-1))
    hs = torch.stack(hiddens, 1)  # [B, T', D]
    for b in range(B):
        e = emb[b * args.text_tokens:(b + 1) * args.text_tokens].reshape(-1, idim).contiguous()
        p = hs[b].reshape(-1, idim).contiguous()
        items.append((e, p))
    first = [None] * B
    last = [None] * B
    samples = [0] * B
    states = []
    for i, seg in speak(engine, items, top_k=args.top_k, min_tokens=args.codec_tokens,
                        max_tokens=args.codec_tokens, states_out=states):
        now = time.perf_counter()  # the segment's length is known on the host: the cut index was read back
        if first[i] is None:
            first[i] = now
        last[i] = now
        samples[i] += seg.numel()
    t_end = time.perf_counter()
    for t in turns:
        t.kv.free()
    stage = {"listen": (t_ss - t_begin) * 1e3, "text": (t_text - t_ss) * 1e3, "speak": (t_end - t_text) * 1e3}
    return dict(t_ss=t_ss, first=first, last=last, samples=samples, first_pcm=[s.t_first_pcm for s in states],
                stage=stage)


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_baseline(cfg_name, threads, seconds_audio, n_chunks, text_tokens, codec_tokens):
    """Oracle (numpy fp32 port of the reference path, oracle/nets.py) timed on host cores at REAL geometry,
    one unit of each kind at FULL depth: U1 = one 160 ms chunk through the 24-block encoder, the adapter
    and all 28 Qwen2 layers + state head; U2 = one text token through the 28 layers + lm_head; U3 = one
    codec token through the 4 AR layers + out_fnn; U4 = one 60-token vocoder call.  Only chunk / token /
    call COUNTS are extrapolated to the turn (no layer extrapolation).  Weights: one random array per
    parameter shape, shared by every layer of that shape (the GEMMs still stream their operands from DRAM:
    each shape's array is far beyond the last-level cache), so the sample needs ~3 GB of host RAM, not
    the 30 GB of distinct fp32 Qwen2 weights.  BLAS threads are set before numpy is imported
    (_blas_threads_from_argv) and verified with threadpoolctl."""
    sys.path.insert(0, ROOT)
    from oracle import configs, nets, params
    cfg = configs.get(cfg_name)
    rng = np.random.default_rng(0)

    class Shared(dict):
        def __init__(self, shapes):
            super().__init__()
            self.shapes, self.by_shape = shapes, {}

        def __missing__(self, k):
            shp = tuple(self.shapes[k])
            pos = k.endswith(("norm.weight", "norm1.weight", "norm2.weight", "layernorm.weight")) or \
                "running_var" in k or "istd" in k
            key = (shp, pos)
            if key not in self.by_shape:
                v = (rng.standard_normal(shp, dtype=np.float32) * np.float32(0.02 if len(shp) > 1 else 0.1))
                self.by_shape[key] = (np.abs(v) + np.float32(1.0)) if pos else v
            self[k] = self.by_shape[key]
            return self[k]

    W = Shared(params.all_shapes(cfg))
    for k in W.shapes:   # generate (and first-touch) every shared array before anything is timed
        W[k]
    try:
        from threadpoolctl import threadpool_info, threadpool_limits
        limiter = threadpool_limits(limits=threads, user_api="blas")
        blas = [d for d in threadpool_info() if d.get("user_api") == "blas"]
        used = max((int(d.get("num_threads", 0)) for d in blas), default=threads)
        blas_lib = ",".join(sorted({d.get("internal_api", "?") for d in blas}))
    except Exception:   # threadpoolctl missing: the env vars set before the numpy import still hold
        limiter, used, blas_lib = None, threads, "unknown"
    try:
        enc, ada = nets.Encoder(W, cfg, "user"), nets.Adapter(W, cfg, "user")
        llm = nets.Qwen2(W, cfg)
        D = cfg["llm"]["hidden_size"]
        feats = rng.standard_normal((19, 80)).astype(np.float32) * 3 + 8
        kv = nets.KV(cfg["llm"]["num_hidden_layers"])
        llm.forward(rng.standard_normal((40, D)).astype(np.float32), kv)   # system prompt context
        est = nets.new_encoder_state(enc.nb)
        ac = None
        enc.infer(feats, est)   # warm (first-touch page faults of the shared arrays)
        t = time.perf_counter()
        e = enc.infer(feats, est)
        a, ac = ada(e, ac)
        h = llm.forward(a, kv)
        nets.state_probs(W, h)
        u1 = time.perf_counter() - t
        t = time.perf_counter()
        h = llm.forward(rng.standard_normal((1, D)).astype(np.float32), kv)
        llm.logits(h)
        u2 = time.perf_counter() - t
        tts = nets.TTSDecoder(W, cfg)
        idim = cfg["decoder_json"][0]
        kvt, P = tts.prefill(rng.standard_normal((32, idim)).astype(np.float32),
                             rng.standard_normal((32, idim)).astype(np.float32))
        tts.step(4, kvt, P)
        t = time.perf_counter()
        n3 = 5
        for i in range(n3):
            tts.step(5 + i, kvt, P)
        u3 = (time.perf_counter() - t) / n3
        codec = nets.Codec(W, cfg)
        t = time.perf_counter()
        codec(rng.integers(0, cfg["codec_json"]["n_codes"], 60))
        u4 = time.perf_counter() - t
    finally:
        if limiter is not None:
            limiter.restore_original_limits()
    n_voc = 1 + max(0, (codec_tokens - 50 + 39) // 40)
    turn = n_chunks * u1 + text_tokens * u2 + codec_tokens * u3 + n_voc * u4
    speak = text_tokens * u2 + codec_tokens * u3 + n_voc * u4
    return {"value": round(seconds_audio / turn, 4), "unit": "x real-time (1 user, 1 turn)", "cores": used,
            "kind": "port",
            "sample": (f"numpy fp32 oracle (oracle/nets.py) at REAL geometry, {used} BLAS threads ({blas_lib}) of "
                       f"{os.cpu_count()} host CPUs ({cpu_model()}); one unit of each kind at full depth (24 encoder "
                       f"blocks, 28 Qwen2 layers, 4 AR layers): U1 chunk {u1 * 1e3:.1f} ms, U2 text token "
                       f"{u2 * 1e3:.1f} ms, U3 codec token {u3 * 1e3:.2f} ms, U4 vocoder {u4 * 1e3:.1f} ms; "
                       f"turn = {n_chunks} U1 + {text_tokens} U2 + {codec_tokens} U3 + {n_voc} U4 for "
                       f"{seconds_audio:.0f} s of speech (counts extrapolated, layers not)"),
            "speak_rtf_per_user": round(seconds_audio / speak, 4),
            "host_cpus": os.cpu_count(), "cpu_model": cpu_model(),
            "units_ms": {"U1": u1 * 1e3, "U2": u2 * 1e3, "U3": u3 * 1e3, "U4": u4 * 1e3}}


def gather_list(dist, vals, world, dev):
    """All ranks' variable-length float lists, concatenated in rank order."""
    import torch
    lt = torch.tensor(vals, dtype=torch.float64, device=dev)
    sizes = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(sizes, torch.tensor([lt.numel()], dtype=torch.int64, device=dev))
    mx = max(int(x) for x in sizes)
    pad = torch.zeros(max(mx, 1), dtype=torch.float64, device=dev)
    pad[:lt.numel()] = lt
    gl = [torch.zeros_like(pad) for _ in range(world)]
    dist.all_gather(gl, pad)
    return [float(v) for g, n in zip(gl, sizes) for v in g[:int(n)].tolist()]


def recorded_traffic(kernel_regex):
    """HBM bytes per launch of the dominant kernel from the newest committed FETCH_SIZE pass of this
    command (profiles/rNN_fetch.json, written by scripts/summarize_profile.py: KiB x 1024 x 2)."""
    import glob
    import re
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_fetch.json")))
    if not files:
        return None, None
    groups = [g for g in json.load(open(files[-1]))["groups"] if re.search(kernel_regex, g["kernel"])]
    if not groups:
        return None, os.path.relpath(files[-1], ROOT)
    g = max(groups, key=lambda g: g["dispatches"])
    return g["hbm_bytes_per_launch"], os.path.relpath(files[-1], ROOT)


def recorded_kernel_avg_us(kernel_regex):
    """Average duration of the dominant kernel in the newest committed rocprofv3 --kernel-trace --stats
    summary (profiles/rNN_kernel_stats.csv, the same bench command under the profiler)."""
    import csv
    import glob
    import re
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_kernel_stats.csv")))
    for f in reversed(files):
        rows = [r for r in csv.DictReader(open(f)) if re.search(kernel_regex, r["Name"])]
        if rows:
            r = max(rows, key=lambda r: int(r["Calls"]))
            return float(r["AverageNs"]) / 1e3, int(r["Calls"]), os.path.relpath(f, ROOT)
    return None, None, None


def gemm_probe(engine, M, reps=2):
    """Average duration of the dominant kernel (Qwen2 gate/up SwiGLU weight stream, the X-stationary
    k_gemm_xs<8,14,1> launch of every layer) with HIP events on the launching stream.
    The launches walk all layers' gate/up weights in order, as a chunk step does, so no launch finds
    its weights in the Infinity Cache from the previous one (273 MB per layer > 256 MB MALL)."""
    import torch
    from fo import _lib, ops
    layers = engine.llm.stack.layers
    L = layers[0]
    x = torch.randn(M, engine.llm.D, device=engine.device)
    out = torch.empty(M, L.gu.N, device=engine.device)
    for Lw in layers[:3]:
        Lw.gu(x, out=out)
    lib = _lib.load()
    import ctypes
    e0, e1 = ctypes.c_void_p(), ctypes.c_void_p()
    lib.fo_event_create(ctypes.byref(e0))
    lib.fo_event_create(ctypes.byref(e1))
    s = ops.stream(engine.device)
    lib.fo_event_record(e0, s)
    n = 0
    for _ in range(reps):
        for Lw in layers:
            Lw.gu(x, out=out)
            n += 1
    lib.fo_event_record(e1, s)
    ms = ctypes.c_float()
    lib.fo_event_elapsed_ms(e0, e1, ctypes.byref(ms))
    lib.fo_event_destroy(e0)
    lib.fo_event_destroy(e1)
    t = ms.value / n / 1e3
    weight_bytes = L.gu.nbytes
    algo = weight_bytes + M * engine.llm.D * 4 + M * L.gu.N * 4
    return {"bytes": algo, "seconds": t, "gbps": algo / t / 1e9, "launches": n}


def duplex_plan(seconds, offset, speech=3.0, silence=1.5, answer=3.75):
    """SURVEY §8(d) config 5 script for one session: the user talks `speech` s, pauses `silence` s, ...;
    the system answers `answer` s from the end of each user IPU, so the user's next IPU barges in at
    silence / answer = 40 % of the answer."""
    user, system = [], []
    t = 0.5 + offset
    while t < seconds:
        user.append((t, t + speech))
        system.append((t + speech, t + speech + answer))
        t += speech + silence
    return user, system


def run_duplex(eng, args, seconds, sync):
    """Config 5 on one replica: args.users duplex sessions (framing B, 224 ms chunks) with scripted VAD,
    system audio re-encoded and prefilled, user barge-in; all sessions' chunks per tick in one batched
    prefill (fo.duplex.DuplexScheduler).  Returns per-tick wall times and counts."""
    from fo.duplex import DuplexScheduler, DuplexSession, ScriptedVAD
    from models.pipeline import inferencePipeline
    pipe = inferencePipeline.from_engine(eng)
    ch = 3584
    n = int(seconds * 16000 / ch)
    sch = DuplexScheduler(pipe)
    chunks = []   # [session][k] -> {identity: s16le bytes}
    for u in range(args.users):
        up, sp = duplex_plan(seconds, 0.224 * u)
        sch.add(DuplexSession(pipe, sid=u, vad={"user": ScriptedVAD(ch, up), "system": ScriptedVAD(ch, sp)}))
        pcm = {"user": synth_pcm(n * ch, 4321 + u), "system": synth_pcm(n * ch, 8765 + u)}
        chunks.append([{i: np.round(pcm[i][k * ch:(k + 1) * ch] * 32767).astype(np.int16).tobytes()
                        for i in ("user", "system")} for k in range(n)])
    sync()
    ticks, counts = [], {"user": 0, "system": 0, "dialog_ss": 0}

    def account(done):
        for _, d, st in done:
            counts[d["identity"]] += 1
            counts["dialog_ss"] += st == "dialog_ss"

    t_all = time.perf_counter()
    for k in range(n):
        # chunk k of both parties arrives for every session; the tick that follows carries the VAD,
        # fbank, gating, serialisation and the batched prefill + state decision (read on the host)
        t = time.perf_counter()
        for u, s in enumerate(sch.sessions):
            for ident in ("user", "system"):
                s.enqueue_audio_data(ident, {"audio": chunks[u][k][ident], "sr": 16000, "enc": "s16le",
                                             "time_stamp": k * ch / 16000.0})
        done = sch.tick()
        ticks.append(time.perf_counter() - t)
        account(done)
    while True:   # features still queued behind the last chunk
        done = sch.tick()
        if not done:
            break
        account(done)
    sync()
    wall = time.perf_counter() - t_all
    for s in sch.sessions:
        s.release()
    return {"wall": wall, "ticks": ticks, "counts": counts, "audio_s": args.users * n * ch / 16000.0}


def main_duplex(args, eng, dev, dist, world, rank, load_s):
    import torch

    def sync():
        torch.cuda.synchronize()

    for _ in range(args.warmup):
        run_duplex(eng, args, 6.0, sync)
    if dist is not None:
        dist.barrier()
    runs = [run_duplex(eng, args, args.duplex_sec, sync) for _ in range(args.steps)]
    wall = sum(r["wall"] for r in runs)
    audio = sum(r["audio_s"] for r in runs)
    ticks = [t * 1e3 for r in runs for t in r["ticks"]]
    if dist is not None:
        t = torch.tensor([wall, audio], dtype=torch.float64, device=dev)
        allw = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(allw, t)
        wall = max(float(x[0]) for x in allw)
        audio = sum(float(x[1]) for x in allw)
        ticks = gather_list(dist, ticks, world, dev)
    if rank == 0:
        c = runs[-1]["counts"]
        line = {
            "metric": "duplex: real-time factor of two-party dialogue audio processed + p50 state-decision latency",
            "value": round(audio / wall, 3),
            "unit": "x real-time (seconds of per-session dialogue per wall second, all sessions)",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(wall / args.steps * 1e3, 2), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "bf16w-fp32a",
            "data": "synthetic (counter-hash weights; synthetic 16 kHz PCM for both parties; scripted VAD)",
            "config": {"workload": f"config 5: {args.users} duplex sessions/GPU x {args.duplex_sec:.0f} s, framing B "
                                   "(224 ms chunks), user 3.0 s speech / 1.5 s pause, system answers 3.75 s, barge-in "
                                   "at 40 %", "users_per_gpu": args.users, "global_users": args.users * world,
                       "parallelism": f"dp{world} (session-pinned replicas)"},
            "p50_decision_ms": round(float(np.percentile(ticks, 50)), 2) if ticks else None,
            "p90_decision_ms": round(float(np.percentile(ticks, 90)), 2) if ticks else None,
            "chunk_period_ms": 224.0,
            "ticks": len(runs[-1]["ticks"]), "user_chunks": c["user"], "system_chunks": c["system"],
            "dialog_ss": c["dialog_ss"], "load_s": round(load_s, 2),
            "roofline": None, "cpu_baseline": None,
        }
        s = json.dumps(line)
        print(s, flush=True)
        if args.out:
            with open(args.out, "w") as f:
                f.write(s + "\n")


def main():
    args = parse()
    import torch
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    # FO_DIST_REHEARSAL=1: the N > 1 path (receive-only replicas, weight broadcast, result gathering) with
    # every rank on cuda:0 over gloo -- a one-GPU rehearsal of what the 8-GPU run does over RCCL
    rehearsal = os.environ.get("FO_DIST_REHEARSAL") == "1"
    if rehearsal:
        local = 0
    if world > 1:
        import torch.distributed as dist
        if rehearsal:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    from fo.engine import FreezeOmniEngine
    model_dir = os.path.join(ROOT, "configs", args.config)
    t0 = time.perf_counter()
    # ranks > 0 allocate the packed layouts without generating or reading weights: rank 0's broadcast fills them
    eng = FreezeOmniEngine(model_dir, device=dev, max_sessions=max(8, args.users), receive_weights=dist is not None
                           and rank > 0)
    torch.cuda.synchronize()
    load_s = time.perf_counter() - t0
    bcast_s = bcast_bytes = None
    weights_verified = None
    if dist is not None:
        # frozen-weight broadcast from rank 0 over RCCL/xGMI (timed separately, excluded from RTF)
        torch.cuda.synchronize()
        dist.barrier()
        tb = time.perf_counter()
        from fo.replica import broadcast_frozen
        bcast_n, bcast_bytes = broadcast_frozen(eng, dist)
        torch.cuda.synchronize()
        bcast_s = time.perf_counter() - tb
        # every replica now holds rank 0's weights, bit for bit (checksums gathered; a mismatch aborts the run)
        from fo.replica import frozen_checksum
        ck = torch.tensor([frozen_checksum(eng)], dtype=torch.int64, device=dev)
        cks = [torch.zeros_like(ck) for _ in range(world)]
        dist.all_gather(cks, ck)
        if len({int(c.item()) for c in cks}) != 1:
            raise RuntimeError(f"frozen weights differ across replicas after the broadcast: {[int(c) for c in cks]}")
        weights_verified = True

    if args.scenario == "duplex":
        main_duplex(args, eng, dev, dist, world, rank, load_s)
        if dist is not None:
            dist.destroy_process_group()
        return

    def sync():
        torch.cuda.synchronize()

    base_kv = eng.system_role("<|im_start|>system\nYou are a helpful assistant.")
    n_samp = int(args.input_sec * 16000)
    users = [rank * args.users + u for u in range(args.users)]
    pcms = [synth_pcm(n_samp, 1234 + u) for u in users]
    for _ in range(args.warmup):
        run_turn(eng, base_kv, pcms, args, sync)
    sync()
    if dist is not None:
        dist.barrier()
    sync()
    t_start = time.perf_counter()
    stats = [run_turn(eng, base_kv, pcms, args, sync) for _ in range(args.steps)]
    sync()
    if dist is not None:
        dist.barrier()
    sync()
    wall = time.perf_counter() - t_start
    sr = 24000.0
    audio = sum(sum(s["samples"]) for s in stats) / sr
    lat = [(f - s["t_ss"]) * 1e3 for s in stats for f in s["first_pcm"] if f is not None]
    lat_gated = [(f - s["t_ss"]) * 1e3 for s in stats for f in s["first"] if f is not None]
    rtf_user = [(n / sr) / (l - s["t_ss"]) for s in stats for n, l in zip(s["samples"], s["last"]) if l is not None]
    # config 2 from the same invocation: one user alone on the replica (1 warm-up turn + 1 timed turn)
    single = None
    if args.users > 1 and not args.no_single_user:
        run_turn(eng, base_kv, pcms[:1], args, sync)
        sync()
        t1 = time.perf_counter()
        s1 = run_turn(eng, base_kv, pcms[:1], args, sync)
        sync()
        w1 = time.perf_counter() - t1
        a1 = s1["samples"][0] / 24000.0
        single = {"workload": "config 2: 1 user on 1 GPU, 10 s input, same turn",
                  "ms_per_turn": round(w1 * 1e3, 2), "value": round(a1 / w1, 3),
                  "first_audio_ms": round((s1["first_pcm"][0] - s1["t_ss"]) * 1e3, 2),
                  "first_emit_gated_ms": round((s1["first"][0] - s1["t_ss"]) * 1e3, 2),
                  "rtf_per_user": round(a1 / (s1["last"][0] - s1["t_ss"]), 3)}
    probe = gemm_probe(eng, 2 * args.users)
    if dist is not None:
        t = torch.tensor([wall, audio], dtype=torch.float64, device=dev)
        allw = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(allw, t)
        wall = max(float(x[0]) for x in allw)
        audio = sum(float(x[1]) for x in allw)
        lat = gather_list(dist, lat, world, dev)
        lat_gated = gather_list(dist, lat_gated, world, dev)
        rtf_user = gather_list(dist, rtf_user, world, dev)
    if rank == 0:
        peak = 8000.0
        # the SwiGLU (last template flag true) M<=16 weight stream: Qwen2 gate/up of every layer
        kre = r"k_gemm_xs<\d+, \d+, 1>"
        traffic, traffic_src = recorded_traffic(kre)
        rp_us, rp_calls, rp_src = recorded_kernel_avg_us(kre)
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            try:
                cpu = cpu_baseline(args.config, args.cpu_threads, args.codec_tokens / 40.0,
                                   int(math.ceil(n_samp / 2560)), args.text_tokens, args.codec_tokens)
            except Exception as e:  # the baseline is reported, never required for the GPU number
                cpu = {"value": None, "unit": "x real-time", "cores": args.cpu_threads, "kind": "port",
                       "sample": f"failed: {type(e).__name__}: {e}"}
        line = {
            "metric": "real-time factor + p50 first-audio-chunk latency, Qwen2-7B, N users/GPU",
            "value": round(audio / wall, 3),
            "unit": "x real-time (aggregate seconds of 24 kHz speech out per wall second)",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(wall / args.steps * 1e3, 2),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "bf16w-fp32a",
            "data": "synthetic (counter-hash weights at Qwen2-7B + paper geometry; synthetic 16 kHz PCM)",
            "config": {"workload": f"config 3: {args.users} users/GPU, {args.input_sec:.0f} s input (160 ms chunks) "
                                   f"+ {args.text_tokens} text tokens + {args.codec_tokens} codec tokens per turn",
                       "model": f"Freeze-Omni ({args.config}): speech encoder + adapter + Qwen2-7B + AR decoder + "
                                "TiCodec", "users_per_gpu": args.users, "global_users": args.users * world,
                       "parallelism": f"dp{world} (session-pinned replicas)"},
            "p50_first_audio_ms": round(float(np.percentile(lat, 50)), 2) if lat else None,
            "p90_first_audio_ms": round(float(np.percentile(lat, 90)), 2) if lat else None,
            "p50_first_emit_gated_ms": round(float(np.percentile(lat_gated, 50)), 2) if lat_gated else None,
            "rtf_per_user_p50": round(float(np.percentile(rtf_user, 50)), 3) if rtf_user else None,
            "load_s": round(load_s, 2), "weight_broadcast_s": None if bcast_s is None else round(bcast_s, 3),
            "weight_broadcast_bytes": bcast_bytes, "weights_verified": weights_verified,
            "roofline": {"bound": "hbm", "achieved": round(probe["gbps"], 1), "peak": peak, "unit": "GB/s",
                         "frac": round(probe["gbps"] / peak, 4),
                         "traffic": None if traffic is None else round(traffic),
                         "traffic_source": traffic_src,
                         "kernel": "k_gemm_xs<8,14,1> (Qwen2 gate/up SwiGLU X-stationary weight stream, M=16, all "
                                   "28 layers in turn)",
                         "bytes_per_launch": probe["bytes"], "avg_launch_us": round(probe["seconds"] * 1e6, 2),
                         "frac_source": "live: HIP events around every layer's gate/up launch on the engine stream "
                                        "(gemm_probe); rocprof_* = the committed rocprofv3 summary of this command",
                         "rocprof_avg_launch_us": None if rp_us is None else round(rp_us, 2),
                         "rocprof_calls": rp_calls,
                         "rocprof_frac": None if rp_us is None else round(probe["bytes"] / (rp_us * 1e-6) / 1e9 / peak, 4),
                         "rocprof_source": rp_src},
            # wall ms per stage of a timed turn (median over the timed turns): listen = 63 chunks through
            # fbank / encoder / adapter / Qwen2 / state head (pipelined), text = dialog_ss -> the last text
            # token's id on the host, speak = TTS prefill + AR decode + vocoder until the last PCM segment
            "stage_ms": {k: round(float(np.median([s["stage"][k] for s in stats])), 2)
                         for k in ("listen", "text", "speak")},
            "single_user": single,
            "cpu_baseline": cpu,
        }
        s = json.dumps(line)
        print(s, flush=True)
        if args.out:
            with open(args.out, "w") as f:
                f.write(s + "\n")
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
