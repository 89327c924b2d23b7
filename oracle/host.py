"""Oracle (TEST INFRASTRUCTURE): streaming emission rules of the speech decoder front end.

find_min_sum_index restates models/decoder/llm2tts.py:70-112; run_chunking restates the 40+10
codec chunking of llm2TTS.run (models/decoder/llm2tts.py:114-160).  numpy, checker only.
"""
import numpy as np

F32 = np.float32


def find_min_sum_index(buffer, syn, N=2401, threshold=0.01):
    """buffer, syn: 1-D float32.  Returns (new_buffer, emitted or None)."""
    arr = np.asarray(syn, F32)
    L = len(arr)
    mid = L // 2
    a = np.abs(arr).astype(np.float64)
    cs = np.concatenate([[0.0], np.cumsum(a)])
    window = (cs[N:] - cs[:-N]) if L >= N else np.zeros(0)
    start = mid - N // 2
    w = window[start:]
    mi = int(np.argmin(w))
    min_sum = w[mi]
    s0 = max(0, mi + start)
    e0 = min(L, mi + N + s0)  # sic: the reference adds the already-updated start (llm2tts.py:98-99)
    min_index = int(np.argmin(np.abs(arr[s0:e0]))) + s0
    if min_sum / N < threshold:
        return arr[min_index:].copy(), np.concatenate([buffer, arr[:min_index]]).astype(F32)
    return np.concatenate([buffer, arr]).astype(F32), None


def post_decode_probs(logits, temperature=1.0, top_k=0, top_p=0.0):
    """The distribution AudioLLM._post_decode draws its token from (models/audioLLM.py:431-477), i.e. the
    `probs` handed to torch.multinomial: softmax(logits / T); top_k > 0 keeps the k largest and
    renormalises; top_p > 0 sorts descending, removes entries whose inclusive cumsum exceeds top_p -- but
    shifts that mask right by one (always keeping the first) only when the first entry alone exceeds
    top_p -- and renormalises.  float32 like the reference; ties keep the lower index."""
    x = np.asarray(logits, F32).reshape(-1)
    if temperature != 1.0:
        x = (x / F32(temperature)).astype(F32)
    e = np.exp((x - x.max()).astype(F32)).astype(F32)
    p = (e / e.sum(dtype=F32)).astype(F32)
    if top_k > 0:
        keep = np.argsort(-p, kind="stable")[:top_k]
        q = np.zeros_like(p)
        q[keep] = p[keep]
        p = (q / q.sum(dtype=F32)).astype(F32)
    if top_p > 0.0:
        order = np.argsort(-p, kind="stable")
        cs = np.cumsum(p[order], dtype=F32)
        remove = cs > F32(top_p)
        if remove[0]:
            remove[1:] = remove[:-1].copy()
            remove[0] = False
        p = p.copy()
        p[order[remove]] = 0
        p = (p / p.sum(dtype=F32)).astype(F32)
    return p


def run_chunking(token_ids, vocoder, codec_chunk_size=40, codec_padding_size=10, N=2401, seg_threshold=0.01,
                 upsample=600):
    """Yield the PCM segments llm2TTS.run emits for a fixed AR token stream; vocoder(ids)->pcm 1-D."""
    left, right = 0, codec_padding_size
    buf = np.zeros(0, F32)
    tok = []
    out = []
    for t in token_ids:
        tok.append(t)
        if len(tok) == left + codec_chunk_size + right:
            syn = vocoder(np.array(tok))
            syn = syn[left * upsample: len(syn) - right * upsample]
            left = codec_padding_size
            tok = tok[-(left + right):]
            buf, seg = find_min_sum_index(buf, syn, N, seg_threshold)
            if seg is not None:
                out.append(seg)
    if len(tok) > 0:
        syn = vocoder(np.array(tok))[left * upsample:]
        out.append(np.concatenate([buf, syn]).astype(F32))
    return out
