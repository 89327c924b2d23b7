#!/usr/bin/env python3
"""Freeze-Omni MI355X benchmark: streaming speech-to-speech turns for N users per GPU.

metric (BASELINE.json): real-time factor + p50 first-audio-chunk latency, Qwen2-7B, N users/GPU.

One "step" = one full dialogue turn for every user on every rank (SURVEY.md §8(d) config 3 per GPU):
  listen : 10 s of synthetic 16 kHz PCM per user streamed in 160 ms chunks (framing A, 63 chunks);
           each chunk = fbank -> speech encoder -> adapter -> Qwen2-7B chunk prefill (per-user paged KV
           forked from a shared system prompt) -> dialog-state head (host read each chunk, as the reference)
  speak  : dialog_ss -> assistant-prefix prefill + 32 text tokens (benchmark policy, SURVEY §8(d): a sentence
           boundary every 8 tokens) -> per sentence, started at its boundary beside the text decode
           (bin/inference.py:152-183): AR speech decoder (EOS masked until 100 codec tokens; 400 = 10 s of
           24 kHz audio per response) -> TiCodec vocoder per 40(+10+10) tokens -> silence-cut emission.
value = seconds of 24 kHz speech emitted by all users on all ranks / max-over-ranks wall seconds
(aggregate real-time factor, higher is better).  Also reported: per-user RTF (audio / (dialog_ss ->
last PCM)), p50/p90 first-audio latency = dialog_ss -> the first segment llm2TTS.run would YIELD, i.e. released by
the find_min_sum_index silence gate (models/decoder/llm2tts.py:141-153, what the reference's caller sees;
random-weight codec output has no 100 ms quiet window, so the gate holds the audio until a sentence's final
flush), and p50_first_pcm_ms = dialog_ss -> PCM of the first vocoder chunk known on the host, before the gate.
Weights: counter-hash synthetic weights at Qwen2-7B / paper geometry (configs/real), generated on
device; no checkpoint is on the box.  `--gpus N` (N > 1) starts N ranks itself (torch.distributed.run, one rank
per GPU, RCCL); under an outer torch.distributed.run each process is one rank and --gpus must equal WORLD_SIZE.
"""
import argparse
import ctypes
import json
import math
import os
import sys
import time


def _blas_threads_from_argv(default=64):
    """--cpu-threads, read before numpy is imported so the BLAS pool is created at that size.  Default 64: one
    socket of the GPU box's 2 x 64-core host (SURVEY §8(d) asks for os.cpu_count() threads or at least a socket);
    the box's cgroup quota admits 16 CPUs of time, which the line states beside the thread count."""
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
    ap.add_argument("--text-tokens", type=int, default=32, help="text tokens per response (bin/inference.py caps 128)")
    ap.add_argument("--sentence-tokens", type=int, default=8,
                    help="benchmark policy: a sentence boundary every N text tokens (SURVEY §8(d))")
    ap.add_argument("--codec-tokens", type=int, default=400, help="codec tokens per response (10 s of 24 kHz speech)")
    ap.add_argument("--no-concurrent-tts", dest="concurrent_tts", action="store_false",
                    help="speak each sentence inside the text loop, as bin/inference.py does (default: a worker "
                         "thread on its own streams, beside the text decode)")
    ap.add_argument("--top-k", type=int, default=1, help="speech decoder top_k (1 = parity/greedy)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pipeline", dest="pipeline", action="store_false",
                    help="listen chunk by chunk (default: encoder stage of chunk c+1 overlaps the LLM of chunk c)")
    ap.add_argument("--listen-chunks", type=int, default=int(os.environ.get("FO_LISTEN_CHUNKS", "8")),
                    help="consecutive 160 ms chunks of the offline input per Qwen2 stage (fo.engine.ListenGroupGraph; "
                         "1: one chunk per stage)")
    ap.add_argument("--scenario", default="turn", choices=["turn", "duplex"],
                    help="turn: config 3 (default, the headline line); duplex: config 5 sessions")
    ap.add_argument("--duplex-sec", type=float, default=60.0, help="duplex: seconds of audio per session")
    ap.add_argument("--cpu-threads", type=int, default=64,
                    help="BLAS threads of the cpu_baseline leg (set before numpy is imported; default one socket)")
    ap.add_argument("--no-single-user", action="store_true", help="skip the config-2 (1 user) leg")
    ap.add_argument("--no-text-ahead", dest="text_ahead", action="store_false",
                    help="read every text step back before queuing the next (default: each step is queued behind the "
                         "previous one with its ids left on the device, TextGraph.launch; a step queued on an EOS draw "
                         "is rolled back and relaunched.  r03u/r03v A/B: text stage 143-147 -> 131-138 ms)")
    ap.add_argument("--no-tts-lane", dest="tts_lane", action="store_false",
                    help="one sentence-speech worker (each sentence in turn on its own streams) instead of the default "
                         "continuously batched speech lane "
                         "(fo.speak.SpeechLane): sentences whose speech overlaps decode in the same AR step; the last "
                         "sentence (started when the text decode is over) speaks on its own streams.  r03zf, four runs "
                         "each on one box: lane 198.3 / 198.5 / 197.9 / 198.6x vs workers 197.5 / 197.2 / 197.6 / "
                         "197.0x (text stage -3.7 ms, speech after the text +1.5 ms)")
    ap.add_argument("--switch-interval", type=float, default=None,
                    help="Python thread switch interval (s) while the sentence-speech worker runs beside the text "
                         "decode (default: the interpreter's 5 ms)")
    ap.add_argument("--out", default=None, help="also write the JSON line to this file")
    ap.add_argument("--launch-selftest", action="store_true", help=argparse.SUPPRESS)
    return ap.parse_args()


def launch_plan(gpus, env, n_visible, argv, script, port):
    """How `bench.py --gpus N` runs (bin/pool.py:61-91: one replica per GPU):
      * ("rank", None): this process is one rank -- N = 1 without a launcher, or a rank started by
        torch.distributed.run (WORLD_SIZE in the environment, which must equal N);
      * ("spawn", cmd): N > 1 and no launcher: start N ranks with torch.distributed.run (one per GPU, RCCL), this
        process only waits for them and exits with their code.  Decided before any GPU call (n_visible comes from
        torch.cuda.device_count(), which does not initialise HIP on this image);
      * ("error", msg): --gpus disagrees with WORLD_SIZE, or N exceeds the visible devices -- one GPU is never
        oversubscribed silently.  FO_DIST_REHEARSAL=1 (every rank on cuda:0 over gloo, labelled as a one-GPU
        rehearsal) is the only way to run N ranks on fewer GPUs."""
    rehearsal = env.get("FO_DIST_REHEARSAL") == "1"
    if "WORLD_SIZE" in env:
        world = int(env["WORLD_SIZE"])
        if world != gpus:
            return "error", f"--gpus {gpus} disagrees with WORLD_SIZE={world} set by the launcher"
        local = int(env.get("LOCAL_RANK", "0"))
        if not rehearsal and local >= n_visible:
            return "error", (f"rank with LOCAL_RANK={local} but only {n_visible} GPU(s) visible "
                             f"(FO_DIST_REHEARSAL=1 runs every rank on cuda:0)")
        return "rank", None
    if gpus < 1:
        return "error", f"--gpus must be >= 1 (got {gpus})"
    if gpus > 1 and not rehearsal and gpus > n_visible:
        return "error", (f"--gpus {gpus} exceeds the {n_visible} visible GPU(s); refusing to put several ranks on one "
                         f"GPU (FO_DIST_REHEARSAL=1 rehearses the N-rank path on cuda:0 over gloo)")
    if gpus == 1:
        return "rank", None
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", script] + list(argv)
    return "spawn", cmd


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch(args):
    """Apply launch_plan for this invocation; returns only in a process that is a rank."""
    import subprocess

    import torch
    # no HIP initialisation on this image: safe before spawning ranks (the selftest never touches a GPU)
    n_visible = args.gpus if args.launch_selftest else torch.cuda.device_count()
    kind, what = launch_plan(args.gpus, os.environ, n_visible, sys.argv[1:], os.path.abspath(__file__),
                             _free_port())
    if kind == "error":
        print(f"bench.py: {what}", file=sys.stderr, flush=True)
        sys.exit(2)
    if kind == "spawn":
        env = dict(os.environ)
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")   # dmabuf IPC only on this pool (RCCL)
        sys.exit(subprocess.call(what, env=env))


def launch_selftest():
    """--launch-selftest: what each rank of a spawned launch sees, without touching a GPU (CPU test of the plumbing):
    ranks join a gloo group, gather (rank, local rank, world, device the rank would pin), rank 0 prints one line."""
    import torch.distributed as dist
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    local = int(os.environ["LOCAL_RANK"])
    dist.init_process_group("gloo")
    got = [None] * world
    dist.all_gather_object(got, {"rank": rank, "local_rank": local, "world": world, "device": f"cuda:{local}",
                                 "master": f"{os.environ['MASTER_ADDR']}:{os.environ['MASTER_PORT']}"})
    if rank == 0:
        print(json.dumps({"launch_selftest": got}), flush=True)
    dist.destroy_process_group()


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
    B = len(pcms)
    t_begin = time.perf_counter()
    turns = [Turn(engine, base_kv, p) for p in pcms]
    fb = engine.fbank("A")
    CH = turns[0].framer.chunk
    n_chunks = int(math.ceil(len(pcms[0]) / CH))
    pipe = engine.listen_pipe(args.listen_chunks) if args.pipeline else None
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
        if pipe is not None and c == 0:
            # the chat prefix comes from the shared-context prefix cache (exact by causality), after which chunk 0
            # is a steady-state chunk: it enters the pipe, so its LLM stage overlaps chunk 1's encoder stage
            items = engine.apply_chat_prefix(items)
            for t, it in zip(turns, items):
                t.enc_cache, t.ada_cache = it["enc_cache"], it["ada_cache"]
        if pipe is not None and (c > 0 or engine._graphable(items)):
            # steady state: this chunk's encoder stage overlaps the previous chunk's LLM stage
            pe_next, _ = pipe.push(items)
            for t, pe in zip(turns, pe_next):
                t.pe = pe
        else:
            for t, r in zip(turns, engine.listen(items)):
                t.enc_cache, t.ada_cache, t.pe = r["enc_cache"], r["ada_cache"], r["pe_index"]
        if c == 0:
            t_c0 = time.perf_counter()   # chunk 0 submitted (pipe) or read back (--no-pipeline)
    if pipe is not None:
        pipe.flush()
    # ---- dialog_ss (benchmark policy forces it at end of input, as bin/inference.py:138 does)
    sync()
    t_ss = time.perf_counter()
    eod = engine.tokenizer.eod_id
    pre = engine.prefix_ids["system"]
    T, S = args.text_tokens, args.sentence_tokens
    n_sent = (T + S - 1) // S
    # 400 codec tokens per response (EOS masked until then), dealt over the sentences
    codec_per = [args.codec_tokens // n_sent + (1 if s < args.codec_tokens % n_sent else 0) for s in range(n_sent)]
    rec = SpeechRecorder(B)
    tts = None
    if args.concurrent_tts:
        tts = LaneTTS(engine, args, rec) if args.tts_lane else SentenceTTS(engine, args, rec)
    text_ids = [[] for _ in turns]
    hiddens = []
    nxt, hid = engine.text_step([(t.kv, pre) for t in turns])
    kvs = [t.kv for t in turns]
    tg = engine.text_graph(kvs, T) if args.text_ahead else None
    pend = None
    s0 = 0
    for j in range(T):
        hiddens.append(hid)
        for b in range(B):
            text_ids[b].append(nxt[b] if nxt[b] != eod else 0)
        if (j + 1) % S == 0 or j == T - 1:
            # sentence boundary (benchmark policy: every S tokens; bin/inference.py:160-173 cuts at punctuation):
            # this sentence's speech starts now, while the text decode goes on (bin/inference.py:82-92)
            job = (hiddens[s0:j + 1], [ids[s0:j + 1] for ids in text_ids], codec_per[len(rec.sentences)],
                   len(rec.sentences))
            rec.sentences.append(time.perf_counter())
            if tts is not None:
                tts.submit(job, last=j == T - 1)
            else:
                run_sentence(engine, args, rec, *job)
            s0 = j + 1
        if j == T - 1:
            break
        if tg is None:
            nxt, hid = engine.text_step([(t.kv, [text_ids[b][-1]]) for b, t in enumerate(turns)])
            continue
        # token j + 1: its step was queued behind step j on step j's draws (still on the device); an EOS draw
        # is fed back as id 0 by this benchmark policy, so such a step is rolled back and relaunched
        if pend is None:
            pend = tg.launch(kvs, [text_ids[b][-1] for b in range(B)])
        elif eod in nxt:
            tg.read(pend)
            for kv in kvs:
                kv.length -= 1
            pend = tg.launch(kvs, [text_ids[b][-1] for b in range(B)])
        cur = pend
        pend = tg.launch(kvs) if j + 2 <= T - 1 else None
        nxt, hid = tg.read(cur)
    t_text = time.perf_counter()   # the last text step's ids were read back: the text stage is done
    if tts is not None:
        tts.join()
    t_end = time.perf_counter()
    for t in turns:
        t.kv.free()
    stage = {"listen": (t_ss - t_begin) * 1e3, "text": (t_text - t_ss) * 1e3, "speak": (t_end - t_ss) * 1e3,
             "speak_after_text": (t_end - t_text) * 1e3, "listen_chunk0": (t_c0 - t_begin) * 1e3}
    for k in sorted(rec.sent_end):   # per sentence: boundary -> speech start (queueing), start -> end
        stage[f"sentence{k}_wait"] = (rec.sent_start[k] - rec.sentences[k]) * 1e3
        stage[f"sentence{k}_speech"] = (rec.sent_end[k] - rec.sent_start[k]) * 1e3
    return dict(t_ss=t_ss, first=rec.first, last=rec.last, samples=rec.samples, first_pcm=rec.first_pcm,
                stage=stage, n_sent=n_sent, codec_tokens=rec.codec_tokens)


class SpeechRecorder:
    """Per-user timing of the speech of one turn, over all its sentences."""

    def __init__(self, B):
        self.first = [None] * B        # first PCM segment released by the silence gate
        self.first_pcm = [None] * B    # first vocoder chunk's PCM known on the host (before the gate)
        self.last = [None] * B
        self.samples = [0] * B
        self.codec_tokens = [0] * B
        self.sentences = []            # host time of each sentence boundary
        self.sent_start = {}           # host time each sentence's speech started / ended (worker side)
        self.sent_end = {}

    def segment(self, i, seg):
        now = time.perf_counter()      # the segment's length is known on the host: the cut index was read back
        if self.first[i] is None:
            self.first[i] = now
        self.last[i] = now
        self.samples[i] += seg.numel()


def sentence_items(engine, hiddens, ids):
    """The sentence's AR-decoder inputs per user (bin/inference.py:82-92): its text-token embeddings and LLM
    hidden rows, each reshaped to [-1, 896] sub-tokens (on the current stream)."""
    import torch
    B, n = len(ids), len(ids[0])
    idim = engine.cfg["decoder_json"][0]
    ids_d = torch.tensor(ids, dtype=torch.int32).to(engine.device)
    emb = engine.llm.embed(ids_d.view(-1))
    hs = torch.stack(hiddens, 1)  # [B, n, D]
    return [(emb[b * n:(b + 1) * n].reshape(-1, idim).contiguous(), hs[b].reshape(-1, idim).contiguous())
            for b in range(B)]


def run_sentence(engine, args, rec, hiddens, ids, n_codec, k=0, stream=None, voc=None):
    """llm2TTS.run for one sentence of every user (bin/inference.py:82-92): the sentence's text-token
    embeddings and LLM hidden rows, each reshaped to [-1, 896] sub-tokens, through the AR decoder (EOS masked
    until n_codec tokens) and the vocoder with silence-cut emission.  stream / voc: the AR
    decode's and the vocoder's streams (None: the engine's own); the inputs are gathered on `stream` too, so
    nothing of the sentence touches the legacy default stream (which would order it against the text decode)."""
    import contextlib

    import torch
    from fo.speak import speak
    rec.sent_start[k] = time.perf_counter()
    with (torch.cuda.stream(stream) if stream is not None else contextlib.nullcontext()):
        items = sentence_items(engine, hiddens, ids)
        states = []
        for i, seg in speak(engine, items, top_k=args.top_k, min_tokens=n_codec, max_tokens=n_codec,
                            states_out=states, stream=stream, voc_stream=voc):
            rec.segment(i, seg)
    rec.sent_end[k] = time.perf_counter()
    for i, st in enumerate(states):
        if rec.first_pcm[i] is None:
            rec.first_pcm[i] = st.t_first_pcm
        rec.codec_tokens[i] += len(st.all_ids)


class LaneTTS:
    """The speech of every sentence on ONE continuously batched lane (fo.speak.SpeechLane) driven by a worker
    thread beside the text decode: a sentence joins the lane's AR decode at its boundary, so sentences whose
    speech overlaps share each decode step (one pass over the decoder's weights) instead of running two decode
    loops side by side.  Each row keeps its own RNG stream, so the ids and PCM are those of SentenceTTS."""

    def __init__(self, engine, args, rec):
        import queue
        import threading
        from fo import ops
        from fo.speak import SpeechLane
        self.err = None
        self.q = queue.Queue()
        stream = ops.engine_stream(engine.device, name="tts")
        voc = ops.engine_stream(engine.device, name="voc")
        pre = ops.engine_stream(engine.device, name="tts1")   # the sentences' prefills, beside the lane's steps
        lane = SpeechLane(engine, top_k=args.top_k, stream=stream, voc_stream=voc, prefill_stream=pre)

        def work():
            import torch
            torch.cuda.set_device(engine.device)
            stop = False
            try:
                while True:
                    while not stop:   # join every sentence that has arrived (wait for one when the lane is idle)
                        try:
                            job = self.q.get(block=lane.idle)
                        except queue.Empty:
                            break
                        if job is None:
                            stop = True
                            break
                        hiddens, ids, n_codec, k = job
                        rec.sent_start[k] = time.perf_counter()
                        with torch.cuda.stream(pre):   # read by the prefill, on the same stream
                            items = sentence_items(engine, hiddens, ids)
                        lane.add(items, n_codec, n_codec, tag=k)
                    if lane.idle:
                        if stop:
                            return
                        continue
                    for i, seg in lane.pump():
                        rec.segment(lane.states[i].key, seg)
                    for k in lane.done_groups:
                        rec.sent_end[k] = time.perf_counter()
                        for st in (s for s in lane.states if s.tag == k):
                            if rec.first_pcm[st.key] is None:
                                rec.first_pcm[st.key] = st.t_first_pcm
                            rec.codec_tokens[st.key] += len(st.all_ids)
                    lane.done_groups.clear()
            except BaseException as e:  # re-raised in the main thread by join()
                self.err = e
            finally:
                lane.free()

        self.t = threading.Thread(target=work, daemon=True)
        self.t.start()
        # the response's last sentence (submitted once the text decode is over) speaks on its own streams beside
        # the lane's remaining rows instead of joining them (two latency-bound steps on two streams overlap; r03v)
        self.tail = SentenceTTS(engine, args, rec, names=("tts2", "voc2"))

    def submit(self, job, last=False):
        if last:
            self.tail.submit(job)
        else:
            self.q.put(job)

    def join(self):
        self.q.put(None)
        self.t.join()
        self.tail.join()
        if self.err is not None:
            raise self.err


class SentenceTTS:
    """The speech of each sentence generated on its own pair of streams (AR decode + vocoder) by a worker
    thread, while the main thread keeps decoding text on the engine stream: a sentence's speech depends only
    on its own text tokens and hidden rows, and the text decode never reads the speech, so the ids and PCM
    are those of the reference's sequential loop (bin/inference.py:152-183, which pauses the text decode for
    each sentence).  Sentences are spoken in order (one user's audio is a sequence).  (Round 3's multi-worker
    mode is gone: the continuously batched lane, LaneTTS, is the default and measured faster, r03zf/zh.)"""

    def __init__(self, engine, args, rec, names=("tts", "voc")):
        import queue
        import threading
        from fo import ops
        self.err = None
        self.q = queue.Queue()
        stream = ops.engine_stream(engine.device, name=names[0])
        voc = ops.engine_stream(engine.device, name=names[1])

        def work():
            import torch
            torch.cuda.set_device(engine.device)
            while True:
                job = self.q.get()
                if job is None:
                    return
                if self.err is None:
                    try:
                        run_sentence(engine, args, rec, *job, stream=stream, voc=voc)
                    except BaseException as e:  # re-raised in the main thread by join()
                        self.err = e

        self.t = threading.Thread(target=work, daemon=True)
        self.t.start()

    def submit(self, job, last=False):
        self.q.put(job)

    def join(self):
        self.q.put(None)
        self.t.join()
        if self.err is not None:
            raise self.err


def vocoder_calls(n, chunk=40, pad=10):
    """Token counts of the vocoder calls llm2TTS.run makes for n codec tokens (models/decoder/llm2tts.py:
    122-160): a call when the buffer holds left + chunk + pad tokens (left 0, then pad), the final flush."""
    calls, left, have = [], 0, 0
    for _ in range(n):
        have += 1
        if have == left + chunk + pad:
            calls.append(have)
            left = pad
            have = left + pad
    if have > 0:
        calls.append(have)
    return calls


def turn_roofline(eng, B, n_chunks, text_tokens, codec_per_sentence, ctx0, bw=8.0e12, mfma=2.5e15,
                  chunks_per_stage=1):
    """Speed-of-light time of one turn's work (each stage against its own bound, the turn as
    Σ max(bytes / HBM BW, flops / dense bf16 MFMA peak)).  Algorithmic bytes: bf16 weights
    streamed once per batched step, the KV read per token at the reference's bf16 (autocast k_proj / v_proj outputs,
    models/pipeline.py:67-68): Qwen2 57,344 B, AR decoder 14,336 B; vocoder as 2*Cin*Cout*K*Tout FLOPs.  This build
    keeps its paged KV in fp32: the bytes that layout reads beyond the bf16 figure are reported apart
    ("kv_fp32_extra_GB"), never counted as work.  ctx0: per-user LLM context when the listen starts (system prompt).
    chunks_per_stage C: the listen's batched step is a group of C chunks (fo.engine.ListenGroupGraph), so its weights
    stream once per group -- ceil(n_chunks / C) times; each chunk still reads its own context.  The one-chunk-per-step
    figure (the reference's schedule, bin/inference.py:106-144) is returned beside it as listen_per_chunk_GB."""
    llm = eng.llm
    kv_llm = llm.stack.n * llm.KVH * llm.hd * 2 * 2
    kv_tts = eng.tts.main.n * eng.tts.H * eng.tts.hd * 2 * 2
    kv_extra = 0.0   # bytes per (algorithmic bf16) KV byte the fp32 layout adds
    w_listen = eng.enc["user"].weight_bytes + eng.ada["user"].weight_bytes + llm.stack.weight_bytes
    rows = 2   # LLM tokens per 160 ms chunk (framing A)
    listen_kv = 0.0
    L = ctx0
    for c in range(n_chunks):
        L += rows + (len(eng.prefix_ids["user"]) if c == 0 else 0)
        listen_kv += B * L * kv_llm
        kv_extra += B * L * kv_llm
    stages = -(-n_chunks // max(1, chunks_per_stage))
    listen_b = stages * w_listen + listen_kv
    listen_one = n_chunks * w_listen + listen_kv
    text_b = 0.0
    L += len(eng.prefix_ids["system"])
    for t in range(text_tokens):
        text_b += llm.stack.weight_bytes + llm.lm_head.nbytes + B * L * kv_llm
        kv_extra += B * L * kv_llm
        L += 1
    speak_b, speak_f = 0.0, 0.0
    pre_w = eng.tts.pre.weight_bytes + eng.tts.main.weight_bytes + (eng.tts.prefix.weight_bytes if eng.tts.prefix else 0)
    for n in codec_per_sentence:
        speak_b += pre_w
        P = 2 * 4 * (text_tokens // max(1, len(codec_per_sentence)))   # prefix + prefill rows (4 sub-tokens each)
        for i in range(n):
            speak_b += eng.tts.weight_bytes_per_step + B * (P + i) * kv_tts
            kv_extra += B * (P + i) * kv_tts
        speak_f += B * sum(eng.codec.flops(T) for T in vocoder_calls(n))
    ms = {"listen": listen_b / bw * 1e3, "text": text_b / bw * 1e3,
          "speak": max(speak_b / bw, 0.0) * 1e3 + speak_f / mfma * 1e3}
    return ms, {"listen_GB": listen_b / 1e9, "listen_stages": stages, "listen_per_chunk_GB": listen_one / 1e9,
                "text_GB": text_b / 1e9, "speak_GB": speak_b / 1e9,
                "vocoder_TFLOP": speak_f / 1e12, "kv_fp32_extra_GB": kv_extra / 1e9}


def codec_ids_check(eng):
    """The product AR decoder + sampler on the reference's real-geometry golden (tests/golden/real_tts_t2.npz:
    LLM2TTSCodecAR.infer at 896 / 14 heads / 4864, 4 layers, top_k = 1, 48 ids; configs/real's weights are the
    golden's).  Returns (matching ids in order, total) -- the codec-token exact match of SURVEY §8(d)."""
    import torch
    from fo.speak import speak
    path = os.path.join(ROOT, "tests", "golden", "real_tts_t2.npz")
    if not os.path.exists(path):
        return None, None
    g = np.load(path)
    items = [(torch.from_numpy(g["hidden"]).to(eng.device), torch.from_numpy(g["prefix"]).to(eng.device))]
    states = []
    for _ in speak(eng, items, top_k=1, max_tokens=len(g["ids"]), states_out=states):
        pass
    got, want = states[0].all_ids, g["ids"].tolist()
    n = 0
    while n < min(len(got), len(want)) and got[n] == want[n]:
        n += 1
    return n, len(want)


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_quota():
    """CPUs this process may use: the cgroup's cpu.max quota (the GPU box grants 16 of its 256), else the
    affinity mask."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            return max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    return len(os.sched_getaffinity(0))


def cpu_baseline(cfg_name, threads, text_tokens, sentence_tokens, codec_tokens):
    """The reference's CPU path restated in numpy fp32 (oracle/nets.py, pinned to the reference's own outputs at
    real geometry by tests/test_oracle_real_qwen2.py and the T2 goldens), timed on this host's cores:
      * config 1 END TO END (bin/inference.py:94-187 on assets/question.wav, top_k = 1): the system-role
        prefill, the 13 framing-A chunks of question.wav (their fbank is the committed fixture
        tests/golden/fbank.npz A_feats, the reference's own features of that file) through the 24-block
        encoder, the adapter, all 28 Qwen2 layers and the state head; dialog_ss: the assistant prefix and
        `text_tokens` greedy text tokens (lm_head over 152,064); per sentence of `sentence_tokens` tokens, the
        AR decoder's prefill and codec tokens (EOS masked, as the GPU bench) and every vocoder call
        llm2TTS.run makes (models/decoder/llm2tts.py:122-160);
      * one unit of each kind at full depth (U1 chunk, U2 text token, U3 codec token, U4 60-token vocoder
        call), and from them the config-2 turn (10 s input) by counts.
    Weights: distinct fp32 arrays for every parameter (copies of one random array per shape: the values do
    not matter for time, distinct memory does -- each layer streams its own ~0.9 GB from DRAM), ~32 GB of
    host RAM.  BLAS threads are set before numpy is imported (_blas_threads_from_argv) and verified with
    threadpoolctl; the cgroup quota is reported beside them."""
    sys.path.insert(0, ROOT)
    from oracle import configs, nets, params
    cfg = configs.get(cfg_name)
    rng = np.random.default_rng(0)
    base = {}

    class Distinct(dict):
        def __init__(self, shapes):
            super().__init__()
            self.shapes = shapes

        def __missing__(self, k):
            shp = tuple(self.shapes[k])
            pos = k.endswith(("norm.weight", "norm1.weight", "norm2.weight", "layernorm.weight")) or \
                "running_var" in k or "istd" in k
            key = (shp, pos)
            if key not in base:
                v = (rng.standard_normal(shp, dtype=np.float32) * np.float32(0.02 if len(shp) > 1 else 0.1))
                base[key] = (np.abs(v) + np.float32(1.0)) if pos else v
            self[k] = base[key].copy()
            return self[k]

    W = Distinct(params.all_shapes(cfg))
    for k in W.shapes:   # materialise (and first-touch) every array before anything is timed
        W[k]
    try:
        from threadpoolctl import threadpool_info, threadpool_limits
        limiter = threadpool_limits(limits=threads, user_api="blas")
        blas = [d for d in threadpool_info() if d.get("user_api") == "blas"]
        used = max((int(d.get("num_threads", 0)) for d in blas), default=threads)
        blas_lib = ",".join(sorted({d.get("internal_api", "?") for d in blas}))
    except Exception:   # threadpoolctl missing: the env vars set before the numpy import still hold
        limiter, used, blas_lib = None, threads, "unknown"
    n_layers = cfg["llm"]["num_hidden_layers"]
    D = cfg["llm"]["hidden_size"]
    idim = cfg["decoder_json"][0]
    n_codes = cfg["codec_json"]["n_codes"]
    try:
        enc, ada = nets.Encoder(W, cfg, "user"), nets.Adapter(W, cfg, "user")
        llm = nets.Qwen2(W, cfg)
        tts = nets.TTSDecoder(W, cfg)
        codec = nets.Codec(W, cfg)
        # ---------------------------------------------------------------- config 1, end to end
        feats = np.load(os.path.join(ROOT, "tests", "golden", "fbank.npz"))["A_feats"]
        n_sent = (text_tokens + sentence_tokens - 1) // sentence_tokens
        per = [codec_tokens // n_sent] * n_sent
        def config1_run():
            t0 = time.perf_counter()
            kv = nets.KV(n_layers)
            V = cfg["llm"]["vocab_size"]

            def emb(ids):   # Qwen2-7B-Instruct chat-template ids (configs.QWEN2_IDS), folded into a smaller vocabulary
                return llm.embed([i % V for i in ids])

            llm.forward(emb(list(range(1, 16))), kv)                    # 'pre': the system role (15 tokens)
            est, ac = nets.new_encoder_state(enc.nb), None
            for c in range(len(feats)):                                 # listen: 13 chunks
                e = enc.infer(feats[c], est)
                a, ac = ada(e, ac)
                if c == 0:
                    a = np.concatenate([emb([151645, 198, 151644, 872, 198]), a])   # user chat prefix
                h = llm.forward(a, kv)
                nets.state_probs(W, h)
            t_listen = time.perf_counter() - t0
            h = llm.forward(emb([151645, 198, 151644, 77091, 198]), kv)   # dialog_ss: assistant prefix
            toks, hids = [], []
            for j in range(text_tokens):
                hids.append(h[-1])
                tok = int(np.argmax(llm.logits(h[-1:])[0]))
                toks.append(tok)
                if j < text_tokens - 1:
                    h = llm.forward(llm.embed([tok]), kv)
            for si in range(n_sent):                                    # speak, sentence by sentence
                sl = slice(si * sentence_tokens, (si + 1) * sentence_tokens)
                kvt, P = tts.prefill(llm.embed(toks[sl]).reshape(-1, idim), np.stack(hids[sl]).reshape(-1, idim))
                cur, ids = tts.vocab + 1, []
                for _ in range(per[si]):
                    lg = tts.step(cur, kvt, P)
                    cur = int(np.argmax(lg[:n_codes]))                  # EOS masked (benchmark policy)
                    ids.append(cur)
                for T in vocoder_calls(per[si]):                     # the calls' token counts (which ids: immaterial)
                    codec(np.asarray(ids[:T]))
            config1 = time.perf_counter() - t0
            return config1, t_listen, kv, est, ac, toks

        config1, t_listen, kv, est, ac, toks = config1_run()
        # ---------------------------------------------------------------- units
        e = enc.infer(feats[0], est)
        t = time.perf_counter()
        e = enc.infer(feats[1], est)
        a, ac = ada(e, ac)
        h = llm.forward(a, kv)
        nets.state_probs(W, h)
        u1 = time.perf_counter() - t
        t = time.perf_counter()
        h = llm.forward(llm.embed([toks[-1]]), kv)
        llm.logits(h)
        u2 = time.perf_counter() - t
        kvt, P = tts.prefill(rng.standard_normal((32, idim)).astype(np.float32),
                             rng.standard_normal((32, idim)).astype(np.float32))
        tts.step(4, kvt, P)
        t = time.perf_counter()
        for i in range(5):
            tts.step(5 + i, kvt, P)
        u3 = (time.perf_counter() - t) / 5
        t = time.perf_counter()
        codec(rng.integers(0, n_codes, 60))
        u4 = time.perf_counter() - t
        # the same config-1 run at the cgroup quota's thread count, when the threads above exceed it (the box
        # admits 16 CPUs of time: 64 BLAS threads there only time-slice, so this is the faster CPU number)
        quota = cpu_quota()
        config1_q = None
        if limiter is not None and quota and quota < used:
            with threadpool_limits(limits=quota, user_api="blas"):
                config1_q = config1_run()[0]
    finally:
        if limiter is not None:
            limiter.restore_original_limits()
    audio1 = codec_tokens * 600 / 24000.0
    n_voc = n_sent * len(vocoder_calls(codec_tokens // n_sent))
    turn2 = 63 * u1 + text_tokens * u2 + codec_tokens * u3 + n_voc * u4
    # the CPU path's best configuration on what the box grants: the faster of the measured thread counts
    best_s, best_threads = config1, used
    if config1_q is not None and config1_q < config1:
        best_s, best_threads = config1_q, quota
    return {"value": round(audio1 / best_s, 4),
            "unit": f"x real-time (config 1: 1 user, question.wav 2.0 s in, {audio1:.0f} s of speech out)",
            "cores": best_threads, "kind": "port",
            "sample": (f"config 1 end to end on the numpy fp32 oracle (oracle/nets.py) at REAL geometry with distinct "
                       f"weights per layer: {len(feats)} question.wav chunks (listen {t_listen:.2f} s at {used} "
                       f"threads), assistant prefix + {text_tokens} text tokens, {n_sent} sentences x {per[0]} codec "
                       f"tokens, {n_voc} vocoder calls = {best_s:.2f} s at {best_threads} BLAS threads ({blas_lib}), "
                       f"the faster of {used} threads ({config1:.2f} s)"
                       + ("" if config1_q is None else f" and the cgroup quota's {quota} ({config1_q:.2f} s)")
                       + f"; host {os.cpu_count()} CPUs ({cpu_model()}), cgroup quota {cpu_quota()} CPUs"),
            "config1_s": round(best_s, 3), "config1_listen_s": round(t_listen, 3),
            "threads_measured": {str(used): round(config1, 3),
                                 **({} if config1_q is None else {str(quota): round(config1_q, 3)})},
            "value_at_socket_threads": round(audio1 / config1, 4),
            "config2_rtf_from_units": round(10.0 / turn2, 4),
            "host_cpus": os.cpu_count(), "cpu_quota": cpu_quota(), "cpu_model": cpu_model(),
            "units_ms": {"U1": round(u1 * 1e3, 2), "U2": round(u2 * 1e3, 2), "U3": round(u3 * 1e3, 3),
                         "U4": round(u4 * 1e3, 2)}}


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
    files = sorted(f for f in glob.glob(os.path.join(ROOT, "profiles", "r*_fetch.json"))
                   if re.fullmatch(r"r\d\d[a-z]*_fetch\.json", os.path.basename(f)))
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
    # only the bench's own summaries (rNN<letter>_kernel_stats.csv), not the AR-step / text-step ones
    files = sorted(f for f in glob.glob(os.path.join(ROOT, "profiles", "r*_kernel_stats.csv"))
                   if re.fullmatch(r"r\d\d[a-z]*_kernel_stats\.csv", os.path.basename(f)))
    for f in reversed(files):
        rows = [r for r in csv.DictReader(open(f)) if re.search(kernel_regex, r["Name"])]
        if rows:
            r = max(rows, key=lambda r: int(r["Calls"]))
            return float(r["AverageNs"]) / 1e3, int(r["Calls"]), os.path.relpath(f, ROOT)
    return None, None, None


def gemm_probe(engine, M, reps=2, down=False):
    """Average duration of the dominant kernel with HIP events on the launching stream: the Qwen2 gate/up SwiGLU
    weight stream of every layer at M rows (M <= 16: the X-stationary k_gemm_xs<16,7>); down=True: the listen group's
    17..64-row split-K stream, which both the gate/up and the down launch (k_gemm_xsk + its k_gemm_reduce): every
    layer's gate/up, then its down, each timed with its reduce (so the reduce counts against the kernel).
    The launches walk all layers' weights in order, as a stage does, so no launch finds its weights in the Infinity
    Cache from the previous one (273 MB per layer > 256 MB MALL)."""
    import torch
    from fo import _lib, ops
    layers = engine.llm.stack.layers
    L = layers[0]
    x = torch.randn(M, engine.llm.D, device=engine.device)
    out = torch.empty(M, L.gu.N, device=engine.device)
    if down:
        xd = torch.randn(M, L.down.K if hasattr(L.down, "K") else L.gu.N, device=engine.device)
        yd = torch.empty(M, engine.llm.D, device=engine.device)
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
            if down:
                Lw.down(xd, out=yd)
                n += 1
    lib.fo_event_record(e1, s)
    ms = ctypes.c_float()
    lib.fo_event_elapsed_ms(e0, e1, ctypes.byref(ms))
    lib.fo_event_destroy(e0)
    lib.fo_event_destroy(e1)
    t = ms.value / n / 1e3
    algo = L.gu.nbytes + M * engine.llm.D * 4 + M * L.gu.N * 4
    if down:   # per launch: the mean of a gate/up and a down launch
        algo = (algo + L.down.nbytes + M * xd.shape[1] * 4 + M * engine.llm.D * 4) / 2
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


def run_duplex(eng, args, seconds, sync, probe=False):
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

    from fo import _lib
    stages = []   # per tick: host gating ms + GPU spans of the batched prefill (engine stage probe)
    t_all = time.perf_counter()
    for k in range(n):
        # chunk k of both parties arrives for every session; the tick that follows carries the VAD,
        # fbank, gating, serialisation and the batched prefill + state decision (read on the host)
        t = time.perf_counter()
        for u, s in enumerate(sch.sessions):
            for ident in ("user", "system"):
                s.enqueue_audio_data(ident, {"audio": chunks[u][k][ident], "sr": 16000, "enc": "s16le",
                                             "time_stamp": k * ch / 16000.0})
        if probe:
            from fo.duplex import deliver_deferred
            defer = []   # the host stages of tick() (VAD, gating + one fbank launch, serialisation), timed apart
            for s in sch.sessions:
                s.pump(defer)
            deliver_deferred(defer)
            t_host = time.perf_counter()
            eng.stage_probe = []
        done = sch.tick()
        ticks.append(time.perf_counter() - t)
        if probe:
            marks, eng.stage_probe = eng.stage_probe, None
            st = {"host_gating": (t_host - t) * 1e3, "items": len(done), "tick": ticks[-1] * 1e3}
            # algorithmic bytes of the tick (SURVEY §8(d) U1 at framing B): each identity's encoder + adapter weights
            # once, the Qwen2 layers once, every prefilled session's KV read at the reference's bf16 (57,344 B a token;
            # the fp32 paged layout's extra half is not work)
            llm = eng.llm
            kv_tok = llm.stack.n * llm.KVH * llm.hd * 2 * 2
            idents = {d["identity"] for _, d, _ in done}
            st["bytes"] = (sum(eng.enc[i].weight_bytes + eng.ada[i].weight_bytes for i in idents) +
                           llm.stack.weight_bytes + sum(ss.past_key_values.get_seq_length() for ss, _, _ in done) * kv_tok)
            for (a, ea, ha), (b, eb, hb) in zip(marks, marks[1:]):
                ms = ctypes.c_float()
                _lib.call("fo_event_elapsed_ms", ea, eb, ctypes.byref(ms))
                st[b] = st.get(b, 0.0) + ms.value
                st["host_" + b] = st.get("host_" + b, 0.0) + (hb - ha) * 1e3   # host time to enqueue the stage
            for _, e, _ in marks:
                _lib.call("fo_event_destroy", e)
            if marks:
                stages.append(st)
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
    return {"wall": wall, "ticks": ticks, "counts": counts, "audio_s": args.users * n * ch / 16000.0,
            "stages": stages}


def dist_info(dist, world):
    """The process group the run used (None: a single process without a launcher)."""
    if dist is None:
        return None
    import torch
    be = dist.get_backend()
    v = None
    if be == "nccl":
        try:
            v = ".".join(str(x) for x in torch.cuda.nccl.version())
        except Exception:
            v = None
    return {"backend": be, "rccl_version": v, "world_size": world}


def topology(world):
    """n_gpus = GPUs the job ran on: a FO_DIST_REHEARSAL run puts every rank on cuda:0, so it is one GPU (its ranks
    are replicas sharing that GPU, not a scaling point)."""
    rehearsal = os.environ.get("FO_DIST_REHEARSAL") == "1"
    return {"n_gpus": 1 if rehearsal else world, "ranks": world, "physical_gpus": 1 if rehearsal else world,
            "rehearsal": "one-GPU rehearsal: every rank on cuda:0 over gloo" if rehearsal else None}


def duplex_stage_split(pr):
    """Median per tick of the probed run, over the ticks that prefilled something: host gating (VAD, fbank, gating,
    serialisation), each identity's encoder + adapter, the LLM input gather, the Qwen2 layers, the state head, and
    the tick's wall time; p50 over the ticks that ran each stage."""
    if not pr:
        return None
    keys = sorted({k for st in pr for k in st if k not in ("items", "bytes")})
    out = {k: round(float(np.median([st[k] for st in pr if k in st])), 3) for k in keys}
    out["ticks_probed"] = len(pr)
    out["items_p50"] = float(np.median([st["items"] for st in pr]))
    return out


def duplex_roofline(pr, eng, bw=8.0e12):
    """The tick against its own bound (config 5): algorithmic bytes of the tick (encoder + adapter
    weights per identity present, Qwen2 layers, KV read) / 8 TB/s vs the tick's wall time, median over probed ticks."""
    if not pr:
        return None
    fr = [st["bytes"] / bw * 1e3 / st["tick"] for st in pr]
    gpu = [st["bytes"] / bw * 1e3 / max(1e-6, sum(v for k, v in st.items() if k in
                                                    ("encoder_user", "encoder_system", "encoders_both", "gather",
                                                     "qwen2", "state_head")))
           for st in pr]
    b = float(np.median([st["bytes"] for st in pr]))
    return {"bound": "hbm", "unit": "GB/s", "peak": 8000.0,
            "achieved": round(b / (float(np.median([st["tick"] for st in pr])) * 1e-3) / 1e9, 1),
            "frac": round(float(np.median(fr)), 4), "frac_gpu_spans": round(float(np.median(gpu)), 4),
            "tick_bytes_p50": round(b), "tick_roofline_ms": round(b / bw * 1e3, 3), "traffic": None,
            "source": "untimed probed run of the same script (engine stage probe); frac = roofline ms / tick wall ms"}


def main_duplex(args, eng, dev, dist, world, rank, load_s):
    import torch

    def sync():
        torch.cuda.synchronize()

    for _ in range(args.warmup):
        run_duplex(eng, args, 6.0, sync)
    if dist is not None:
        dist.barrier()
    runs = [run_duplex(eng, args, args.duplex_sec, sync) for _ in range(args.steps)]
    # untimed: the same script with the per-tick stage probe (HIP events on the engine stream, host gating timed
    # apart) -- the split and the tick roofline come from here, the headline numbers from the runs above
    pr = run_duplex(eng, args, min(args.duplex_sec, 30.0), sync, probe=True)["stages"]
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
            **topology(world), "steps": args.steps, "warmup": args.warmup,
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
            "roofline": duplex_roofline(pr, eng),
            "tick_stage_ms": duplex_stage_split(pr),
            "dist": dist_info(dist, world),
            "cpu_baseline": None,
        }
        s = json.dumps(line)
        print(s, flush=True)
        if args.out:
            with open(args.out, "w") as f:
                f.write(s + "\n")


def main():
    args = parse()
    launch(args)   # --gpus N > 1 without a launcher: spawns N ranks and exits with their code
    if args.launch_selftest:
        launch_selftest()
        return
    if args.switch_interval:
        sys.setswitchinterval(args.switch_interval)
    import torch
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    # FO_DIST_REHEARSAL=1: the N > 1 path (receive-only replicas, weight broadcast, result gathering) with
    # every rank on cuda:0 over gloo -- a one-GPU rehearsal of what the 8-GPU run does over RCCL; its line says
    # physical_gpus 1 and n_gpus 1 (the ranks are replicas sharing one GPU, not a scaling point)
    rehearsal = os.environ.get("FO_DIST_REHEARSAL") == "1"
    if rehearsal:
        local = 0
    # every torch.distributed.run rank joins the process group, at world 1 too: the launcher path, RCCL init, the
    # weight broadcast and the checksum all_gather are one code path whatever N is
    launched = "WORLD_SIZE" in os.environ and "RANK" in os.environ
    if world > 1 or launched:
        import torch.distributed as dist
        if rehearsal:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    if world > 1:
        # N ranks on one node: no rank's host loop fans a large CPU tensor op over a 16-thread OpenMP pool (whose
        # spinning threads, N times over, can exhaust a CPU quota and stall every rank's ticks: r05z); the engine's
        # host code needs no intra-op parallelism (same rate at 1 thread at N = 1, profiles/r05zb_omp_threads_ab.txt)
        torch.set_num_threads(1)
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
                  "first_audio_ms": round((s1["first"][0] - s1["t_ss"]) * 1e3, 2),
                  "first_pcm_ms": round((s1["first_pcm"][0] - s1["t_ss"]) * 1e3, 2),
                  "rtf_per_user": round(a1 / (s1["last"][0] - s1["t_ss"]), 3)}
    # the dominant kernel by time in the turn (r06v rocprof: 12.9 % of kernel time): the text steps' gate/up SwiGLU at
    # `users` rows (k_gemm_xs, 33 steps x 28 layers), ahead of the grouped listen's gate/up (k_gemm_rows at
    # 2 x users x C rows, 8 stages x 28 layers: 6.4 %), which is reported beside it (listen_kernel)
    group_rows = 2 * args.users * args.listen_chunks if args.pipeline else 2 * args.users
    probe = gemm_probe(eng, args.users)
    probe_l = gemm_probe(eng, group_rows, down=16 < group_rows <= 64) if group_rows > 16 else None
    codec_ok, codec_n = codec_ids_check(eng)
    n_chunks = int(math.ceil(n_samp / 2560))
    roof_ms, roof_units = turn_roofline(eng, args.users, n_chunks, args.text_tokens,
                                        [args.codec_tokens // stats[0]["n_sent"]] * stats[0]["n_sent"], base_kv.length,
                                        chunks_per_stage=args.listen_chunks if args.pipeline else 1)
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
        # the X-stationary SwiGLU M<=16 weight stream: Qwen2 gate/up of every layer (the shipped variant: template
        # VAR 0, spelled out in the kernel name since round 5; the probe variants 1-4 never run in the bench); with
        # listen groups of 17..64 rows the split-K stream of their gate/up and down, RB = ceil(rows / 16)
        rb = (group_rows + 15) // 16
        kre = r"k_gemm_xs<\d+, \d+(, 0)?>"
        kname = (f"k_gemm_xs<16,7> (Qwen2 gate/up SwiGLU X-stationary weight stream, M={args.users}: the text steps, "
                 f"all 28 layers in turn)")
        if group_rows <= 64:
            kre_l = rf"k_gemm_xsk<\d+, \d+, {rb}, \d+>"
            kname_l = (f"k_gemm_xsk<8,KPW,{rb},UA> + its k_gemm_reduce (the listen group's Qwen2 gate/up SwiGLU and "
                       f"down split-K weight streams, M={group_rows}; per launch = the mean of a gate/up and a down)")
        else:
            kre_l = r"k_gemm_rows<8, 1, 30,"
            kname_l = (f"k_gemm_rows<8,1,30,2,2> + its k_gemm_reduce (the listen group's Qwen2 gate/up SwiGLU weight "
                       f"stream at M={group_rows}: 8 waves split the rows, the weight fragments shared through an "
                       f"LDS-DMA ring, K in thirds; all 28 layers in turn, reduce included)")
        traffic, traffic_src = recorded_traffic(kre)
        rp_us, rp_calls, rp_src = recorded_kernel_avg_us(kre)
        listen_kernel = None
        if probe_l is not None:
            tr_l, _ = recorded_traffic(kre_l)
            rl_us, rl_calls, _ = recorded_kernel_avg_us(kre_l)
            listen_kernel = {"kernel": kname_l, "achieved": round(probe_l["gbps"], 1), "unit": "GB/s",
                             "frac": round(probe_l["gbps"] / 8000.0, 4), "bytes_per_launch": probe_l["bytes"],
                             "avg_launch_us": round(probe_l["seconds"] * 1e6, 2),
                             "traffic": None if tr_l is None else round(tr_l),
                             "rocprof_avg_launch_us": None if rl_us is None else round(rl_us, 2),
                             "rocprof_calls": rl_calls}
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            try:
                cpu = cpu_baseline(args.config, args.cpu_threads, args.text_tokens, args.sentence_tokens,
                                   args.codec_tokens)
            except Exception as e:  # the baseline is reported, never required for the GPU number
                cpu = {"value": None, "unit": "x real-time", "cores": args.cpu_threads, "kind": "port",
                       "sample": f"failed: {type(e).__name__}: {e}"}
        line = {
            "metric": "real-time factor + p50 first-audio-chunk latency, Qwen2-7B, N users/GPU",
            "value": round(audio / wall, 3),
            "unit": "x real-time (aggregate seconds of 24 kHz speech out per wall second)",
            **topology(world), "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(wall / args.steps * 1e3, 2),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "bf16w-fp32a",
            "data": "synthetic (counter-hash weights at Qwen2-7B + paper geometry; synthetic 16 kHz PCM)",
            "config": {"workload": f"config 3: {args.users} users/GPU, {args.input_sec:.0f} s input (160 ms chunks) "
                                   f"+ {args.text_tokens} text tokens in {stats[0]['n_sent']} sentences of "
                                   f"{args.sentence_tokens} + {args.codec_tokens} codec tokens per turn "
                                   f"({args.codec_tokens // stats[0]['n_sent']} per sentence); each sentence's speech "
                                   + ("starts at its boundary beside the text decode" if args.concurrent_tts else
                                      "runs inside the text loop (bin/inference.py order)"),
                       "text_tokens": args.text_tokens, "sentences": stats[0]["n_sent"],
                       "codec_tokens": args.codec_tokens, "listen_chunks_per_stage": args.listen_chunks,
                       "model": f"Freeze-Omni ({args.config}): speech encoder + adapter + Qwen2-7B + AR decoder + "
                                "TiCodec", "users_per_gpu": args.users, "global_users": args.users * world,
                       "parallelism": f"dp{world} (session-pinned replicas)"},
            # first audio = the first segment llm2TTS.run yields, after find_min_sum_index's gate
            # (models/decoder/llm2tts.py:141-153); first PCM = the first vocoder chunk on the host, before the gate
            "p50_first_audio_ms": round(float(np.percentile(lat_gated, 50)), 2) if lat_gated else None,
            "p90_first_audio_ms": round(float(np.percentile(lat_gated, 90)), 2) if lat_gated else None,
            "p50_first_pcm_ms": round(float(np.percentile(lat, 50)), 2) if lat else None,
            "p90_first_pcm_ms": round(float(np.percentile(lat, 90)), 2) if lat else None,
            "rtf_per_user_p50": round(float(np.percentile(rtf_user, 50)), 3) if rtf_user else None,
            "load_s": round(load_s, 2), "weight_broadcast_s": None if bcast_s is None else round(bcast_s, 3),
            "weight_broadcast_bytes": bcast_bytes, "weights_verified": weights_verified,
            "dist": dist_info(dist, world),
            "roofline": {"bound": "hbm", "achieved": round(probe["gbps"], 1), "peak": peak, "unit": "GB/s",
                         "frac": round(probe["gbps"] / peak, 4),
                         "traffic": None if traffic is None else round(traffic),
                         "traffic_source": traffic_src,
                         "kernel": kname,
                         "bytes_per_launch": probe["bytes"], "avg_launch_us": round(probe["seconds"] * 1e6, 2),
                         "frac_source": "live: HIP events around every layer's gate/up launch on the engine stream "
                                        "(gemm_probe); rocprof_* = the committed rocprofv3 summary of this command "
                                        "(split-K kernels: the stream kernel alone, its reduce not included)",
                         "listen_kernel": listen_kernel,
                         "rocprof_avg_launch_us": None if rp_us is None else round(rp_us, 2),
                         "rocprof_calls": rp_calls,
                         "rocprof_frac": None if rp_us is None else round(probe["bytes"] / (rp_us * 1e-6) / 1e9 / peak, 4),
                         "rocprof_source": rp_src,
                         # the whole turn against its speed of light: Σ over the turn's units of
                         # max(bytes / 8 TB/s, FLOPs / 2.5 PF) vs the measured ms per turn, and each stage vs its
                         # own wall window (text and speak overlap: speak's window starts at dialog_ss too)
                         "turn_roofline_ms": round(sum(roof_ms.values()), 2),
                         "turn_frac": round(sum(roof_ms.values()) / (wall / args.steps * 1e3), 4),
                         "stages": {k: {"ms": round(float(np.median([s["stage"][k] for s in stats])), 2),
                                        "roofline_ms": round(roof_ms[k], 2),
                                        "frac": round(roof_ms[k] / float(np.median([s["stage"][k] for s in stats])), 4)}
                                    for k in ("listen", "text", "speak")},
                         "units": {k: round(v, 3) for k, v in roof_units.items()}},
            "codec_ids_exact": {"matched": codec_ok, "total": codec_n,
                                "source": "tests/golden/real_tts_t2.npz (reference LLM2TTSCodecAR.infer, top_k=1, "
                                          "real geometry, the bench's own decoder weights)"},
            # wall ms per stage of a timed turn (median over the timed turns): listen = 63 chunks through
            # fbank / encoder / adapter / Qwen2 / state head (pipelined), text = dialog_ss -> the last text
            # token's id on the host, speak = TTS prefill + AR decode + vocoder until the last PCM segment
            # (+ per sentence: boundary -> its speech starting on the worker, and that speech's duration)
            "stage_ms": {k: round(float(np.median([s["stage"][k] for s in stats])), 2)
                         for k in stats[0]["stage"]},
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
