"""speechEncoder (reference: models/encoder/encoder.py:45-155) over fo.speech.SpeechEncoderEngine.

Constructed the reference's way -- speechEncoder(input_dim, overview_conf, para_conf, global_cmvn), the
train.yaml encoder_conf dicts and a GlobalCMVN (models/encoder/cmvn.py) -- it builds its own engine with
counter-hash synthetic weights under the reference's parameter names (the CMVN statistics from
global_cmvn), and load_state_dict(sd) re-packs it from a reference state dict (global_cmvn.*, enc.0.*,
enc.1.* keys).  The reference re-parses sys.argv inside its constructor (encoder.py:54-57); this one reads
only the dicts it is given.  speechEncoder(engine) is the encoder of an existing engine (AudioLLM).

infer(xs_pad, buffer, buffer_index, buffer_out, pe_index) keeps the reference signature; `buffer` is an
opaque fo.speech.EncoderCache (pass None / the reference's [None]*num_blocks list to start)."""
import collections

import torch

_Keys = collections.namedtuple("IncompatibleKeys", ["missing_keys", "unexpected_keys"])


class _TransformerView:
    def __init__(self, nb):
        self.num_blocks = nb


class speechEncoder:
    IDENT = "user"   # the engine's parameter prefix: encoder_user.*

    def __init__(self, input_dim, overview_conf=None, para_conf=None, global_cmvn=None, *, device="cuda:0", seed=0,
                 max_sessions=64):
        from fo.speech import SpeechEncoderEngine
        if isinstance(input_dim, SpeechEncoderEngine):   # the encoder of an existing engine (AudioLLM)
            self._cfg = None
            self._set_engine(input_dim)
            return
        if not torch.cuda.is_available():
            raise RuntimeError("speechEncoder needs an MI355X (gfx950) device: there is no CPU fallback")
        if overview_conf is None or para_conf is None:
            raise ValueError("speechEncoder: overview_conf and para_conf (train.yaml encoder_conf) are required")
        layers = overview_conf.get("encoder-layer-config", "subsampling-transformer").split("-")
        if layers != ["subsampling", "transformer"]:
            raise ValueError(f"speechEncoder: encoder-layer-config {overview_conf.get('encoder-layer-config')!r}: the "
                             "streaming infer path is subsampling-transformer (models/encoder/encoder.py:149-155)")
        tr = para_conf["transformer"]
        if tr.get("transformer-pos-enc-class", "rel-enc") != "rel-enc" or \
                tr.get("transformer-positionwise-layer-type", "linear") != "linear":
            raise ValueError("speechEncoder: only rel-enc positions and linear FFNs have a streaming infer "
                             "(models/encoder/attention.py:7-68,105,254-266)")
        self._cfg = {"train_yaml": {"input_dim": int(input_dim),
                                    "encoder_conf": {"overview_conf": dict(overview_conf), "para_conf": para_conf}}}
        self._device, self._max_sessions = torch.device(device), max_sessions
        from fo.params import encoder_shapes
        from fo.weights import CheckpointSource, OverlaySource, SynthSource
        self._shapes = encoder_shapes(self._cfg, self.IDENT)
        self._synth = SynthSource(seed, self._shapes, self._device)
        self.global_cmvn = global_cmvn
        # CMVN is folded into the first im2col (models/encoder/cmvn.py:24-35); without a GlobalCMVN the
        # reference normalises nothing (encoder.py:149-152), i.e. mean 0 / istd 1
        idim = self._shapes[f"encoder_{self.IDENT}.global_cmvn.mean"][0]
        mean = torch.zeros(idim) if global_cmvn is None else torch.as_tensor(global_cmvn.mean).float().cpu()
        istd = torch.ones(idim) if global_cmvn is None else torch.as_tensor(global_cmvn.istd).float().cpu()
        p = f"encoder_{self.IDENT}.global_cmvn."
        src = OverlaySource(CheckpointSource({p + "mean": mean.reshape(-1), p + "istd": istd.reshape(-1)}, self._device),
                            self._synth)
        self._base = src
        self._set_engine(self._build(src))

    def _build(self, src):
        from fo.speech import SpeechEncoderEngine
        return SpeechEncoderEngine(src, self._cfg, self.IDENT, self._device, self._max_sessions)

    def _set_engine(self, engine):
        self.engine = engine
        self.enc = [None, _TransformerView(engine.nb)]

    def output_size(self):
        return self.engine.d

    def state_dict_shapes(self):
        """The reference module's state-dict keys and shapes (models/encoder/encoder.py:45-99)."""
        if self._cfg is None:
            raise RuntimeError("speechEncoder(engine): the weights belong to the engine (load them through it)")
        p = f"encoder_{self.IDENT}."
        return {k[len(p):]: tuple(v) for k, v in self._shapes.items()}

    def load_state_dict(self, state_dict, strict=True):
        """Re-pack the encoder from a reference state dict (tensors or arrays keyed like the reference module)."""
        from fo.weights import CheckpointSource, OverlaySource
        shapes = self.state_dict_shapes()
        unexpected = [k for k in state_dict if k not in shapes]
        # the reference registers global_cmvn's buffers only when it was given one (encoder.py:60)
        missing = [k for k in shapes if k not in state_dict and (self.global_cmvn is not None
                                                                   or not k.startswith("global_cmvn."))]
        bad = [f"{k}: {tuple(torch.as_tensor(v).shape)} != {shapes[k]}" for k, v in state_dict.items()
               if k in shapes and tuple(torch.as_tensor(v).shape) != shapes[k]]
        if bad:
            raise RuntimeError("speechEncoder.load_state_dict: size mismatch: " + "; ".join(bad))
        if strict and (unexpected or missing):
            raise RuntimeError(f"speechEncoder.load_state_dict: missing {missing[:8]}, unexpected {unexpected[:8]}")
        p = f"encoder_{self.IDENT}."
        state = {p + k: torch.as_tensor(v).detach().float().cpu() for k, v in state_dict.items() if k in shapes}
        self._set_engine(self._build(OverlaySource(CheckpointSource(state, self._device), self._base)))
        return _Keys(missing, unexpected)

    def infer(self, xs_pad, buffer, buffer_index=0, buffer_out=None, pe_index=0):
        cache = buffer if hasattr(buffer, "slot") else self.engine.new_cache()
        feats = torch.as_tensor(xs_pad).to(self.engine.device, torch.float32)
        feats = feats.reshape(-1, feats.shape[-2], feats.shape[-1]).contiguous()
        out, T, pes = self.engine.infer(feats, [cache], [pe_index])
        return out.view(1, T, -1), cache, buffer_index, buffer_out, pes[0]
