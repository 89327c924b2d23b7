"""Host-side logic of the drop-in layer, checked on CPU (no GPU calls)."""
import copy
import json
import os

import numpy as np
import pytest
import torch

from oracle import configs as OC
from oracle import params as OP
from oracle import weights as OW

G = os.path.join(os.path.dirname(__file__), "golden")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_post_process_matches_reference_golden():
    from models.pipeline import inferencePipeline
    g = json.load(open(os.path.join(G, "text_and_serializer.json")))
    for t, want in zip(g["texts"], g["post_process"]):
        assert inferencePipeline.post_process(None, t) == want, t


def test_context_serializer_matches_reference_golden():
    from models.ContextSerializer import ContextSerializer
    g = json.load(open(os.path.join(G, "text_and_serializer.json")))
    cs = ContextSerializer()
    for i, (ts, ident, st) in enumerate(g["events"]):
        cs.add_feature_chunk({"time_stamp": ts, "identity": ident, "status": st, "feature": [i], "ipu_id": i})
    got = []
    while cs.feature_queue:
        got.append(cs.get_next_feature())
    assert got == g["serialized"]


@pytest.mark.parametrize("name", ["tiny", "real"])
def test_param_inventory_and_init_spec_match_oracle(name):
    from fo import params as FP
    from fo import weights as FW
    cfg = OC.get(name)
    a, b = FP.all_shapes(cfg), OP.all_shapes(cfg)
    assert a == b
    for k, shp in b.items():
        assert tuple(FW.init_spec(k, tuple(shp), cfg["overrides"])) == tuple(OW.init_spec(k, tuple(shp),
                                                                                        cfg["overrides"])), k
        assert FW.tensor_key(cfg["seed"], k) == OW.tensor_key(cfg["seed"], k)


@pytest.mark.parametrize("name", ["tiny", "real"])
def test_model_dirs_in_sync_with_configs(name, tmp_path):
    OC.write_model_dirs(OC.get(name), str(tmp_path))
    for rel in ("audiollm/train.yaml", "decoder/model.json", "codec/model.json", "synthetic.json", "llm/config.json"):
        assert open(os.path.join(tmp_path, rel)).read() == open(os.path.join(ROOT, "configs", name, rel)).read(), rel


def test_engine_config_loader_reads_reference_layout():
    from fo.engine import load_model_dir
    cfg, synth, llm_path = load_model_dir(os.path.join(ROOT, "configs", "real"))
    assert cfg["llm"]["hidden_size"] == 3584 and cfg["decoder_json"][0] == 896
    assert synth["seed"] == OC.REAL["seed"] and llm_path.endswith("llm")
    assert cfg["train_yaml"]["encoder_conf"]["para_conf"]["transformer"]["transformer-num-blocks"] == 24


def test_byte_fallback_tokenizer_roundtrip_and_chat_specials():
    from fo.tokenizer import ByteFallbackTokenizer
    t = ByteFallbackTokenizer()
    ids = t.encode("<|im_start|>system\nYou are 你好.<|im_end|>")
    assert ids[0] == 151644 and ids[-1] == 151645
    assert t.decode(ids) == "<|im_start|>system\nYou are 你好.<|im_end|>"
    assert t(["<|im_end|>"])["input_ids"][0][0] == 151645
    assert all(i < 152064 for i in ids)
    # the chat template encodes to Qwen2-7B-Instruct's own ids (and lengths): the benchmark's prefills
    # have the real prompt sizes
    tpl = "<|im_start|>system\nYou are a helpful assistant.<|im_end|>\n<|im_start|>user\n"
    assert t.encode(tpl) == [151644, 8948, 198, 2610, 525, 264, 10950, 17847, 13, 151645, 198, 151644, 872, 198]
    assert t.encode("<|im_end|>\n<|im_start|>assistant\n") == [151645, 198, 151644, 77091, 198]
    assert t.decode(t.encode(tpl)) == tpl


def test_tiny_tokenizer_chat_template_ids_match_reference():
    from fo.tokenizer import load_tokenizer
    meta = json.load(open(os.path.join(G, "audiollm_tiny.json")))
    tok = load_tokenizer(os.path.join(ROOT, "configs", "tiny", "llm"), 384)
    assert tok("<|im_end|>")["input_ids"][0] == meta["eod_id"]
    assert tok(["<|im_start|>system\nYou are a helpful assistant."])["input_ids"][0] == meta["role_ids"]


def test_cmvn_loaders(tmp_path):
    from models.encoder.cmvn import load_cmvn
    rng = np.random.default_rng(0)
    x = rng.standard_normal((500, 80)) * 3 + 5
    js = {"mean_stat": x.sum(0).tolist(), "var_stat": (x ** 2).sum(0).tolist(), "frame_num": 500}
    p = tmp_path / "cmvn.json"
    p.write_text(json.dumps(js))
    m, istd = load_cmvn(str(p), True)
    np.testing.assert_allclose(m, x.mean(0), rtol=1e-9)
    np.testing.assert_allclose(istd, 1 / x.std(0), rtol=1e-6)
    k = tmp_path / "global_cmvn"
    k.write_text("[ " + " ".join(map(str, js["mean_stat"])) + " 500 \n " + " ".join(map(str, js["var_stat"])) + " 0 ]")
    m2, i2 = load_cmvn(str(k), False)
    np.testing.assert_allclose(m2, m, rtol=1e-9)
    np.testing.assert_allclose(i2, istd, rtol=1e-6)


def test_paged_kv_cow_fork_and_free():
    from fo.kv import BatchMeta, KVPool, KVSeq
    pool = KVPool(2, 1, 4, 16, 4, "cpu")
    base = KVSeq(pool)
    BatchMeta([(base, 6, 0, True)], "cpu")       # 6 tokens: 1 full page + partial page
    assert base.length == 6 and len(base.pages) == 2
    pool.k[:, base.pages[1]] = 7.0
    a, b = base.fork(), base.fork()
    assert pool.ref[base.pages[0]] == 3 and pool.pages_in_use() == 2
    m = BatchMeta([(a, 3, 6, True), (b, 1, 6, True)], "cpu")
    assert a.pages[0] == base.pages[0]                 # full page stays shared
    assert a.pages[1] != base.pages[1] and b.pages[1] != base.pages[1]   # partial page copied on write
    assert torch.all(pool.k[:, a.pages[1]] == 7.0)
    assert m.tok_nvis.tolist() == [7, 8, 9, 7] and m.tok_pos.tolist() == [6, 7, 8, 6]
    assert m.tok_slot[0].item() == a.pages[1] * 4 + 2
    assert m.last_rows_host == [2, 3] and m.block_table.shape == (2, 3)
    a.free()
    b.free()
    base.free()
    assert pool.pages_in_use() == 0


def test_batch_meta_rows_match_per_token_rule():
    """BatchMeta's per-token rows (sequence, RoPE position, cache slot, visible keys) follow the per-token rule for
    ragged batches of short (filled token by token) and long (filled vectorised, > 8 tokens) entries, causal and
    full, from arbitrary starting lengths across page boundaries."""
    import numpy as np
    from fo.kv import BatchMeta, KVPool, KVSeq
    pool = KVPool(1, 1, 4, 512, 16, "cpu")
    for trial in range(12):
        rng = np.random.default_rng(trial)
        seqs = [KVSeq(pool) for _ in range(5)]
        for s in seqs:
            s.reserve(int(rng.integers(0, 40)))
            s.length = len(s.pages) * 16 - int(rng.integers(0, 16)) if s.pages else 0
        ents = [(s, int(rng.integers(1, 40)), int(rng.integers(0, 9)), bool(rng.integers(0, 2))) for s in seqs]
        olds = [s.length for s in seqs]
        m = BatchMeta(ents, "cpu", gqa=2)
        rows = []
        for k, (s, n, p0, causal) in enumerate(ents):
            rows += [(k, p0 + i, s.slot(olds[k] + i), olds[k] + i + 1 if causal else olds[k] + n) for i in range(n)]
        got = list(zip(m.tok_seq.tolist(), m.tok_pos.tolist(), m.tok_slot.tolist(), m.tok_nvis.tolist()))
        assert got == rows
        for s in seqs:
            s.free()


def test_pastkv_deepcopy_forks():
    from fo.kv import KVPool, KVSeq, BatchMeta
    from models.audioLLM import PastKeyValues
    pool = KVPool(1, 1, 4, 8, 4, "cpu")
    s = KVSeq(pool)
    BatchMeta([(s, 5, 0, True)], "cpu")
    p = PastKeyValues(s)
    q = copy.deepcopy(p)
    assert q.get_seq_length() == 5 and q.seq is not s and q.seq.pages == s.pages
