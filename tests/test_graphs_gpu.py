"""Captured listen step (fo.engine.ListenGraph) against the eager launch sequence."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(__file__), "golden")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def eng(dev):
    from fo.engine import FreezeOmniEngine
    return FreezeOmniEngine(os.path.join(ROOT, "configs", "tiny"), device=dev, max_sessions=16)


def _session_run(eng, feats_seq, graph, n_users):
    base = eng.system_role("<|im_start|>system\nYou are a helpful assistant.")
    kvs = [base.fork() for _ in range(n_users)]
    state = [dict(enc_cache=None, ada_cache=None, pe_index=0) for _ in range(n_users)]
    out = []
    for c, f in enumerate(feats_seq):
        items = [dict(identity="user", status="ipu_sl" if c == 0 else "ipu_cl", feats=f[u], kv=kvs[u], **state[u])
                 for u in range(n_users)]
        res = eng.listen(items, graph=graph)
        for u, r in enumerate(res):
            state[u] = dict(enc_cache=r["enc_cache"], ada_cache=r["ada_cache"], pe_index=r["pe_index"])
        h, row = res[0]["hidden_row"]
        out.append(([(r["probs"]["state_1"], r["probs"]["state_2"]) for r in res],
                    [h[rr].cpu().numpy().copy() for rr in [r["hidden_row"][1] for r in res]],
                    [kv.length for kv in kvs], [r["pe_index"] for r in res]))
    for kv in kvs:
        kv.free()
    base.free()
    return out


def test_listen_graph_matches_eager(eng, dev):
    g = np.load(os.path.join(G, "fbank.npz"))
    n_users = 3
    feats = torch.from_numpy(g["A_feats"]).to(dev)          # [13, 19, 80]
    seq = [torch.stack([feats[(c + 4 * u) % 13] for u in range(n_users)]) for c in range(7)]
    eager = _session_run(eng, seq, False, n_users)
    graph = _session_run(eng, seq, True, n_users)
    assert len(eng._lgraphs) >= 1                             # the graph path really ran
    for (pe, he, le, qe), (pg, hg, lg, qg) in zip(eager, graph):
        assert le == lg and qe == qg
        np.testing.assert_allclose(np.array(pg), np.array(pe), atol=1e-5)
        for a, b in zip(hg, he):
            np.testing.assert_allclose(a, b, atol=2e-5, rtol=1e-5)


def _session_pipe(eng, feats_seq, n_users, first_in_pipe=False):
    """Chunk 0 through listen() (chat prefix), the rest through a ListenPipe; first_in_pipe: chunk 0 too, after
    engine.apply_chat_prefix (the bench's order)."""
    base = eng.system_role("<|im_start|>system\nYou are a helpful assistant.")
    kvs = [base.fork() for _ in range(n_users)]
    state = [dict(enc_cache=None, ada_cache=None, pe_index=0) for _ in range(n_users)]
    out = []
    pipe = eng.listen_pipe()

    def record(res):
        out.append(([(r["probs"]["state_1"], r["probs"]["state_2"]) for r in res],
                    [r["hidden_row"][0][r["hidden_row"][1]].cpu().numpy().copy() for r in res],
                    None, [r["pe_index"] for r in res]))

    for c, f in enumerate(feats_seq):
        items = [dict(identity="user", status="ipu_sl" if c == 0 else "ipu_cl", feats=f[u], kv=kvs[u], **state[u])
                 for u in range(n_users)]
        if c == 0 and first_in_pipe:
            items = eng.apply_chat_prefix(items)
            for u, it in enumerate(items):
                state[u] = dict(enc_cache=it["enc_cache"], ada_cache=it["ada_cache"], pe_index=it["pe_index"])
        elif c == 0:
            res = eng.listen(items)
            for u, r in enumerate(res):
                state[u] = dict(enc_cache=r["enc_cache"], ada_cache=r["ada_cache"], pe_index=r["pe_index"])
            record(res)
            continue
        pe_next, prev = pipe.push(items)
        for u in range(n_users):
            state[u]["pe_index"] = pe_next[u]
        if prev is not None:
            record(prev)
    record(pipe.flush())
    lens = [kv.length for kv in kvs]
    for kv in kvs:
        kv.free()
    base.free()
    return out, lens


@pytest.mark.parametrize("first_in_pipe", [False, True])
def test_listen_pipe_matches_sequential(eng, dev, first_in_pipe):
    """Encoder stage of chunk c+1 overlapped with the LLM stage of chunk c gives the sequential results; with
    first_in_pipe chunk 0 (its chat prefix from the shared-context prefix cache) enters the pipe too."""
    g = np.load(os.path.join(G, "fbank.npz"))
    n_users = 3
    feats = torch.from_numpy(g["A_feats"]).to(dev)
    seq = [torch.stack([feats[(c + 5 * u) % 13] for u in range(n_users)]) for c in range(9)]
    ref = _session_run(eng, seq, True, n_users)
    got, lens = _session_pipe(eng, seq, n_users, first_in_pipe)
    assert len(got) == len(ref)
    assert lens == ref[-1][2]
    for (pe, he, _, qe), (pg, hg, _, qg) in zip(ref, got):
        assert qe == qg
        np.testing.assert_array_equal(np.array(pg), np.array(pe))
        for a, b in zip(hg, he):
            np.testing.assert_array_equal(a, b)


def test_listen_pipe_decide_stops_and_rolls_back(eng, dev):
    """decide(results of chunk c-1) returning False (dialog_ss) rolls back chunk c's speculatively queued LLM
    stage: the context holds exactly the chunks before it, and the states seen match the sequential run's."""
    g = np.load(os.path.join(G, "fbank.npz"))
    n_users = 2
    feats = torch.from_numpy(g["A_feats"]).to(dev)
    seq = [torch.stack([feats[(c + 3 * u) % 13] for u in range(n_users)]) for c in range(8)]
    ref = _session_run(eng, seq[:5], True, n_users)           # chunks 0..4
    base = eng.system_role("<|im_start|>system\nYou are a helpful assistant.")
    kvs = [base.fork() for _ in range(n_users)]
    state = [dict(enc_cache=None, ada_cache=None, pe_index=0) for _ in range(n_users)]
    seen = []

    def decide(res):
        seen.append([(r["probs"]["state_1"], r["probs"]["state_2"]) for r in res])
        return len(seen) < 4                                  # stop after the decision on chunk 4

    pipe = eng.listen_pipe()
    for c, f in enumerate(seq):
        items = [dict(identity="user", status="ipu_sl" if c == 0 else "ipu_cl", feats=f[u], kv=kvs[u], **state[u])
                 for u in range(n_users)]
        if c == 0:
            for u, r in enumerate(eng.listen(items)):
                state[u] = dict(enc_cache=r["enc_cache"], ada_cache=r["ada_cache"], pe_index=r["pe_index"])
            continue
        pe, _ = pipe.push(items, decide)
        for u in range(n_users):
            state[u]["pe_index"] = pe[u]
        if pipe.stopped:
            break
    assert pipe.stopped and c == 5 and pipe.flush() is None
    assert [kv.length for kv in kvs] == ref[-1][2]             # chunk 5 never reached the context
    for (pe_ref, _, _, _), pg in zip(ref[1:], seen):
        np.testing.assert_array_equal(np.array(pg), np.array(pe_ref))
    with pytest.raises(RuntimeError):
        pipe.push(items)
    for kv in kvs:
        kv.free()
    base.free()


def _group_pipe(eng, feats_seq, n_users, C, decide=None):
    """The bench's order (chunk 0 after apply_chat_prefix, then every chunk through the pipe) with C chunks per
    Qwen2 stage; returns the per-chunk results in order and the final KV lengths."""
    base = eng.system_role("<|im_start|>system\nYou are a helpful assistant.")
    kvs = [base.fork() for _ in range(n_users)]
    state = [dict(enc_cache=None, ada_cache=None, pe_index=0) for _ in range(n_users)]
    out = []
    pipe = eng.listen_pipe(C)

    def record(groups):
        for res in groups or []:
            out.append(([(r["probs"]["state_1"], r["probs"]["state_2"]) for r in res],
                        [r["hidden_row"][0][r["hidden_row"][1]].cpu().numpy().copy() for r in res],
                        [r["pe_index"] for r in res]))

    for c, f in enumerate(feats_seq):
        items = [dict(identity="user", status="ipu_sl" if c == 0 else "ipu_cl", feats=f[u], kv=kvs[u], **state[u])
                 for u in range(n_users)]
        if c == 0:
            items = eng.apply_chat_prefix(items)
            for u, it in enumerate(items):
                state[u] = dict(enc_cache=it["enc_cache"], ada_cache=it["ada_cache"], pe_index=it["pe_index"])
        pe_next, prev = pipe.push(items, decide)
        for u in range(n_users):
            state[u]["pe_index"] = pe_next[u]
        record([prev] if C == 1 and prev is not None else prev)
        if pipe.stopped:
            break
    if not pipe.stopped:
        last = pipe.flush()
        record([last] if C == 1 and last is not None else last)
    lens = [kv.length for kv in kvs]
    for kv in kvs:
        kv.free()
    base.free()
    return out, lens, c


@pytest.mark.parametrize("C,n_chunks", [(2, 9), (4, 10), (3, 3)])
def test_listen_group_pipe_matches_one_chunk_per_stage(eng, dev, C, n_chunks):
    """C consecutive chunks per Qwen2 stage (fo.engine.ListenGroupGraph, the offline input's listen): every chunk's
    state probabilities (1e-4) and last hidden row (1e-3, the oracle-parity bound) equal the one-chunk-per-stage
    pipe's (the encoder and Qwen2 GEMMs tile C x the rows), its pe_index and the context lengths exactly; a partial
    last group (n_chunks % C) is flushed."""
    g = np.load(os.path.join(G, "fbank.npz"))
    n_users = 3
    feats = torch.from_numpy(g["A_feats"]).to(dev)
    seq = [torch.stack([feats[(c + 5 * u) % 13] for u in range(n_users)]) for c in range(n_chunks)]
    ref, lens_ref, _ = _group_pipe(eng, seq, n_users, 1)
    got, lens, _ = _group_pipe(eng, seq, n_users, C)
    assert len(got) == len(ref) == n_chunks and lens == lens_ref
    worst = 0.0
    for (pr, hr, qr), (pg, hg, qg) in zip(ref, got):
        assert qr == qg
        # (the batched-vs-single bound of tests/test_duplex_gpu.py: the two pipes' graphs tile the Qwen2 stage and its
        # attention splits differently)
        np.testing.assert_allclose(np.array(pg), np.array(pr), atol=1e-4)
        for a, b in zip(hg, hr):
            # (the grouped encoder and Qwen2 stage run their norms and GEMMs over C x the rows: other kernels, other fp32
            # summation orders, amplified through the encoder and Qwen2 blocks; test_grouped_encoder_pass_equals_chunk_by_
            # chunk holds the encoder alone to 2e-5.  The bound is the oracle-parity tolerance of these rows,
            # tests/test_parity_r02_gpu.py: atol 1e-3)
            worst = max(worst, float(np.abs(a - b).max()))
            np.testing.assert_allclose(a, b, atol=1e-3, rtol=1e-4)
    print(f"[listen group C={C}] worst hidden-row deviation {worst:.2e} abs")


def test_listen_group_pipe_decide_rolls_back_the_rest(eng, dev):
    """A refusal on chunk 4 (the second chunk of group 2 at C = 3; group 3 already queued) leaves exactly chunks
    0..4 in the context, as the one-chunk pipe's refusal does."""
    g = np.load(os.path.join(G, "fbank.npz"))
    n_users = 2
    feats = torch.from_numpy(g["A_feats"]).to(dev)
    seq = [torch.stack([feats[(c + 3 * u) % 13] for u in range(n_users)]) for c in range(12)]
    seen = []

    def decide(res):
        seen.append(1)
        return len(seen) < 5     # refuse chunk 4
    got, lens, last = _group_pipe(eng, seq, n_users, 3, decide)
    ref, lens_ref, _ = _group_pipe(eng, seq[:5], n_users, 1)
    assert len(got) == 5 and lens == lens_ref
    for (pr, _, qr), (pg, _, qg) in zip(ref, got):
        assert qr == qg
        np.testing.assert_allclose(np.array(pg), np.array(pr), atol=1e-4)


def _text_run(eng, graph, n_users, steps, top_k):
    base = eng.system_role("<|im_start|>system\nYou are a helpful assistant.")
    kvs = [base.fork() for _ in range(n_users)]
    pre = eng.prefix_ids["system"]
    ids, hid = eng.text_step([(kv, pre) for kv in kvs], top_k=top_k, seed=7)   # prefix: eager either way
    out = [(list(ids), hid.cpu().numpy().copy())]
    for _ in range(steps):
        ids, hid = eng.text_step([(kv, [i]) for kv, i in zip(kvs, ids)], top_k=top_k, seed=7, graph=graph)
        out.append((list(ids), hid.cpu().numpy().copy()))
    lens = [kv.length for kv in kvs]
    for kv in kvs:
        kv.free()
    base.free()
    return out, lens


@pytest.mark.parametrize("top_k", [1, 5])
def test_text_graph_matches_eager(eng, top_k):
    """The captured text-decode step (fo.engine.TextGraph) draws the same ids as the eager step (same
    kernels and counter RNG), with the same hidden rows and KV lengths."""
    eager, le = _text_run(eng, False, 3, 12, top_k)
    graph, lg = _text_run(eng, True, 3, 12, top_k)
    assert len(eng._tgraphs) >= 1 and le == lg
    for (ie, he), (ig, hg) in zip(eager, graph):
        assert ie == ig
        np.testing.assert_allclose(hg, he, atol=2e-5, rtol=1e-5)


@pytest.mark.parametrize("top_k", [1, 5])
def test_text_graph_launch_ahead_matches_step_by_step(eng, top_k):
    """TextGraph.launch without ids (the step queued behind the previous one, fed by its draws on the device)
    gives the step-by-step graph path's ids, hidden rows and KV lengths exactly -- including a step rolled back
    and relaunched with host ids (what bench.py's --text-ahead does when a draw must be replaced)."""
    ref, lr = _text_run(eng, True, 3, 12, top_k)
    base = eng.system_role("<|im_start|>system\nYou are a helpful assistant.")
    kvs = [base.fork() for _ in range(3)]
    pre = eng.prefix_ids["system"]
    ids, hid = eng.text_step([(kv, pre) for kv in kvs], top_k=top_k, seed=7)
    out = [(list(ids), hid.cpu().numpy().copy())]
    tg = eng.text_graph(kvs, 12, top_k=top_k, seed=7)
    pend = tg.launch(kvs, ids)
    for j in range(12):
        if j == 5:   # roll the queued step back and relaunch it from the host's ids (the same ones here)
            tg.read(pend)
            for kv in kvs:
                kv.length -= 1
            pend = tg.launch(kvs, out[-1][0])
        cur = pend
        pend = tg.launch(kvs) if j < 11 else None
        ids, hid = tg.read(cur)
        out.append((list(ids), hid.cpu().numpy().copy()))
    assert [kv.length for kv in kvs] == lr
    for (ir, hr), (ig, hg) in zip(ref, out):
        assert ir == ig
        np.testing.assert_array_equal(hg, hr)
    for kv in kvs:
        kv.free()
    base.free()


def test_shared_context_prefix_cache_matches_uncached(eng, dev):
    """First chunk (ipu_sl, chat prefix) of sessions forked from one system role: the cached prefix KV
    (computed once, each session a copy-on-write fork of it, the chunk then a captured steady-state step)
    gives the state probs, hidden rows and KV lengths of the per-session prefill that appends the prefix rows
    in the chunk's own forward (models/audioLLM.py:404-419), and later chunks agree too."""
    g = np.load(os.path.join(G, "fbank.npz"))
    n_users = 3
    feats = torch.from_numpy(g["A_feats"]).to(dev)
    seq = [torch.stack([feats[(c + 5 * u) % 13] for u in range(n_users)]) for c in range(4)]
    eng.use_prefix_cache = False
    try:
        plain = _session_run(eng, seq, True, n_users)
    finally:
        eng.use_prefix_cache = True
    n0 = len(eng._prefix_kv)
    cached = _session_run(eng, seq, True, n_users)
    assert len(eng._prefix_kv) >= max(1, n0)                  # the cache really served chunk 0
    for (pp, hp, lp, qp), (pc, hc, lc, qc) in zip(plain, cached):
        assert lp == lc and qp == qc
        np.testing.assert_allclose(np.array(pc), np.array(pp), atol=2e-5)
        for a, b in zip(hc, hp):
            np.testing.assert_allclose(a, b, atol=5e-5, rtol=1e-5)
