"""TiCodec vocoder (VQVAE.forward) on the MI355X kernels, batched over sessions.

Reference: models/decoder/ticodec/vqvae.py:37-42 (quantizer.embed + embed_gst + generator),
models/decoder/ticodec/models.py:59-166 (ResBlock1/2), :169-242 (Generator.forward).
"""
import ctypes
import os
from types import SimpleNamespace

import torch

from . import _lib, ops
from .ops import F32, I32


class CodecEngine:
    MAX_GRAPHS = 32

    def __init__(self, src, codec_json, device):
        h = self.h = codec_json
        self.device = torch.device(device)
        assert h["residul_layer"] == 1 and h["n_code_groups"] == 1, "single-codebook TiCodec only (the speech decoder emits one id per frame)"
        self.codebook = src.get("codec.quantizer.quantizer_modules.0.embedding.weight", torch.bfloat16)
        gt = h["global_tokens"]
        # embed_gst's tables (models.py:703-715), one per global token: row t of table j is that token's slice
        self.gst_tables = [src.get(f"codec.quantizer.quantizer_modules_globaltokens.{j}.embedding.weight").contiguous()
                           for j in range(len(gt))]
        parts = [tab[t] for tab, t in zip(self.gst_tables, gt)]
        self.gfeat = torch.cat(parts).contiguous()  # [128]: the configured voice (h.global_tokens), the default
        p = "codec.generator."
        g = lambda n, dt=F32: src.get(p + n, dt)  # noqa: E731
        self.U = h["upsample_initial_channel"]
        self.conv_pre = (g("conv_pre.weight", torch.bfloat16), g("conv_pre.bias"))
        self.ups = [(g(f"ups.{i}.weight", torch.bfloat16), g(f"ups.{i}.bias"), u, k)
                    for i, (u, k) in enumerate(zip(h["upsample_rates"], h["upsample_kernel_sizes"]))]
        nk = len(h["resblock_kernel_sizes"])
        self.res = []
        for i in range(len(self.ups)):
            stage = []
            for j, (k, dil) in enumerate(zip(h["resblock_kernel_sizes"], h["resblock_dilation_sizes"])):
                r = f"resblocks.{i * nk + j}."
                if h["resblock"] == "1":
                    convs = [((g(r + f"convs1.{m}.weight", torch.bfloat16), g(r + f"convs1.{m}.bias"), d),
                              (g(r + f"convs2.{m}.weight", torch.bfloat16), g(r + f"convs2.{m}.bias"), 1))
                             for m, d in enumerate(dil)]
                else:
                    convs = [((g(r + f"convs.{m}.weight", torch.bfloat16), g(r + f"convs.{m}.bias"), d), None)
                             for m, d in enumerate(dil)]
                stage.append((k, convs))
            self.res.append(stage)
        self.conv_post = (g("conv_post.weight", torch.bfloat16), g("conv_post.bias"))
        self.upsample = 1
        for u in h["upsample_rates"]:
            self.upsample *= u
        # MFMA path: every conv packed once into A-fragment order (fo_vocoder.hip)
        self.p_pre = ops.PackedConv(*self.conv_pre)
        self.p_ups = []
        for w, b, u, k in self.ups:
            pad = (k - u) // 2
            phases = []
            for r in range(u):
                j0 = (r + pad) % u
                pc = ops.PackedConv(w, b, transposed=(j0, u))
                off = (r + pad - j0) // u
                phases.append((r, pc, pc.K - 1 - off))  # (phase, weights, pad of the equivalent conv)
            self.p_ups.append(phases)
        self.use_graphs = os.environ.get("FO_CODEC_GRAPH", "1") != "0"
        # ResBlock1 stages as grouped launches (fo_conv_cl_multi): the u polyphase components of each upsampling
        # in one launch, the stage's resblock chains side by side (one launch per conv position), their last
        # convs summed into the stage output by one launch -- 7 launches a stage instead of u + 18.
        # FO_CODEC_GROUPED=0: one launch per conv (A/B)
        # and the narrow stages' (16 / 32 / 64 channels) two convs of a ResBlock1 step in one workgroup
        # (fo_conv_pair_multi), FO_CODEC_PAIR=0 to keep them apart (A/B)
        self.pair = os.environ.get("FO_CODEC_PAIR", "1") != "0"
        self.grouped = (h["resblock"] == "1" and os.environ.get("FO_CODEC_GROUPED", "1") != "0"
                        and len({len(c) for _, c in self.res[0]}) == 1 and len(self.res[0]) <= 5
                        and max(h["upsample_rates"]) <= 5)
        self._graphs = {}   # (B, T, stream) -> static buffers (+ captured graph), least recently used first
        self.p_res = [[(k, [(ops.PackedConv(c1[0], c1[1]), c1[2], None if c2 is None else ops.PackedConv(c2[0], c2[1]))
                            for c1, c2 in convs]) for k, convs in stage] for stage in self.res]

    def flops(self, T):
        """Algorithmic FLOPs of one generator call on T tokens (2*Cin*Cout*K*Tout per conv)."""
        f = 2 * 512 * self.U * 7 * T
        C, L = self.U, T
        for i, (w, b, u, k) in enumerate(self.ups):
            Co = C // 2
            f += 2 * C * Co * k * L  # transposed conv: every input sample meets k taps
            L *= u
            C = Co
            for k2, convs in self.res[i]:
                f += sum(2 * C * C * k2 * L * (2 if c2 is not None else 1) for _, c2 in convs)
        f += 2 * C * 7 * L
        return f

    def _buffers(self, B, T):
        """Static activations of one (B, T) call: every conv reads and writes these, so the call can be
        captured once as a hipGraph and replayed."""
        dev, F = self.device, dict(dtype=F32, device=self.device)
        E = self.codebook.shape[1]
        bufs = SimpleNamespace(B=B, T=T, exec=None, ids=torch.empty(B, T, dtype=I32, device=dev),
                               x0=torch.empty(B, T, E, **F), y0=torch.empty(B, T, self.U, **F),
                               g=self.gfeat.view(1, -1).expand(B, -1).contiguous(), stages=[])
        C, L = self.U, T
        for w, b, u, k in self.ups:
            C, L = C // 2, (L - 1) * u - 2 * ((k - u) // 2) + k
            nb = len(self.res[0]) if self.grouped else 1   # one chain's buffers per resblock
            bufs.stages.append(SimpleNamespace(C=C, L=L, up=torch.empty(B, L, C, **F),
                                               t1=[torch.empty(B, L, C, **F) for _ in range(nb)],
                                               ya=[torch.empty(B, L, C, **F) for _ in range(nb)],
                                               yb=[torch.empty(B, L, C, **F) for _ in range(nb)],
                                               xs=torch.empty(B, L, C, **F)))
        bufs.out = torch.empty(B, L, **F)
        return bufs

    def _run(self, bf):
        """The generator on bf's buffers.  ResBlock1 (models.py:59-110) chains y = y + c2(leaky(c1(leaky(y))))
        over the dilations; the last conv of resblock j writes xs = (xs + y + c2) directly, and the last
        resblock's scales by 1/num_kernels and adds the global-token feature (models.py:229-238), so the
        stage has no clone / axpy / scale passes."""
        B, T = bf.B, bf.T
        E = self.codebook.shape[1]
        ops.codec_embed_cl(self.codebook, E, self.codebook.shape[0], bf.ids, B, T, bf.x0)
        ops.conv_cl(bf.x0, B, E, T, self.p_pre, 1, 3, bf.y0)
        x, C, L = bf.y0, self.U, T
        for i, (w, b, u, k) in enumerate(self.ups):
            S = bf.stages[i]
            if self.grouped:   # leaky -> ConvTranspose1d as u polyphase convs, one launch
                ops.conv_cl_multi([ops.conv_desc(x, L, pc, 1, pad_r, S.up, Tq=(S.L - r + u - 1) // u, ostride=u, ooff=r,
                                                 Tout_total=S.L, pre_leaky=0.1) for r, pc, pad_r in self.p_ups[i]],
                                  B, C, S.C, self.device)
            else:
                for r, pc, pad_r in self.p_ups[i]:  # leaky -> ConvTranspose1d as u polyphase convs
                    Tq = (S.L - r + u - 1) // u
                    ops.conv_cl(x, B, C, L, pc, 1, pad_r, S.up, Tq=Tq, ostride=u, ooff=r, Tout_total=S.L,
                                pre_leaky=0.1)
            C, L = S.C, S.L
            nk = len(self.p_res[i])
            gadd = bf.g if C == bf.g.shape[1] else None
            if self.grouped:
                self._stage_grouped(S, B, C, L, self.p_res[i], gadd)
                x = S.xs
                continue
            for j, (kk, convs) in enumerate(self.p_res[i]):
                src, last_j = S.up, j == nk - 1
                for m, (p1, d1, p2) in enumerate(convs):
                    if m == len(convs) - 1:
                        dst, res2 = S.xs, (S.xs if j > 0 else None)
                        osc, ga = (1.0 / nk, gadd) if last_j else (1.0, None)
                    else:
                        dst, res2, osc, ga = (S.ya[0] if src is not S.ya[0] else S.yb[0]), None, 1.0, None
                    if p2 is None:  # ResBlock2: y = y + conv(leaky(y))
                        ops.conv_cl(src, B, C, L, p1, d1, (kk * d1 - d1) // 2, dst, pre_leaky=0.1, res=src, res2=res2,
                                    oscale=osc, gadd=ga)
                    else:
                        ops.conv_cl(src, B, C, L, p1, d1, (kk * d1 - d1) // 2, S.t1[0], pre_leaky=0.1)
                        ops.conv_cl(S.t1[0], B, C, L, p2, 1, (kk - 1) // 2, dst, pre_leaky=0.1, res=src, res2=res2,
                                    oscale=osc, gadd=ga)
                    src = dst
            x = S.xs
        w, b = self.conv_post
        ops.conv_post_cl(x, B, L, C, w, b, w.shape[-1], (w.shape[-1] - 1) // 2, 0.1, bf.out)

    def _stage_grouped(self, S, B, C, L, res, gadd):
        """The stage's ResBlock1 chains side by side (models.py:59-110, 221-238): for each dilation position m,
        one launch of every chain's c1 and one of every chain's c2 (y_j = y_j + c2(leaky(c1(leaky(y_j))))); the
        last c2 launch sums the chains into xs = (sum_j y_j) / num_kernels + g, so no chain's partial sum is
        ever stored."""
        dev, nk, nd = self.device, len(res), len(res[0][1])
        src = [S.up] * nk
        if self.pair and C in ops.PAIR_CHANNELS:
            # narrow late stages: both convs of a step in one workgroup (fo_conv_pair_multi), c1's output in LDS
            for m in range(nd):
                last = m == nd - 1
                dst = [S.xs] * nk if last else [S.ya[j] if src[j] is not S.ya[j] else S.yb[j] for j in range(nk)]
                ops.conv_pair_multi([(src[j], res[j][1][m][0], res[j][1][m][2], res[j][0], res[j][1][m][1], dst[j])
                                     for j in range(nk)], B, C, L, dev, summed=last,
                                    oscale=1.0 / nk if last else 1.0, gadd=gadd if last else None)
                src = dst
            return
        for m in range(nd):
            ops.conv_cl_multi([ops.conv_desc(src[j], L, res[j][1][m][0], res[j][1][m][1],
                                             (res[j][0] * res[j][1][m][1] - res[j][1][m][1]) // 2, S.t1[j],
                                             pre_leaky=0.1) for j in range(nk)], B, C, C, dev)
            if m < nd - 1:
                dst = [S.ya[j] if src[j] is not S.ya[j] else S.yb[j] for j in range(nk)]
                ops.conv_cl_multi([ops.conv_desc(S.t1[j], L, res[j][1][m][2], 1, (res[j][0] - 1) // 2, dst[j],
                                                 pre_leaky=0.1, res=src[j]) for j in range(nk)], B, C, C, dev)
                src = dst
            else:
                ops.conv_cl_multi([ops.conv_desc(S.t1[j], L, res[j][1][m][2], 1, (res[j][0] - 1) // 2, S.xs,
                                                 pre_leaky=0.1, res=src[j], oscale=1.0 / nk, gadd=gadd)
                                   for j in range(nk)], B, C, C, dev, summed=True)

    def global_feature(self, gst, B):
        """embed_gst (models/decoder/ticodec/models.py:703-715) of per-call global style tokens: gst int [Bg, 1, n] or
        [Bg, n] (VQVAE.encode's layout; Bg = B, or 1 broadcast over the batch) -> device fp32 [B, n * d], each row the
        concatenation of table j's row gst[b, j] (fo_gather_rows per table into its column slice)."""
        n, d = len(self.gst_tables), self.gst_tables[0].shape[1]
        g = torch.as_tensor(gst).reshape(-1, n)
        if g.shape[0] not in (1, B):
            raise ValueError(f"global_style_token batch {g.shape[0]} does not match the codes' batch {B}")
        hi = min(int(t.shape[0]) for t in self.gst_tables)
        gh = g.cpu()
        if int(gh.min()) < 0 or int(gh.max()) >= hi:   # nn.Embedding raises IndexError on such ids
            raise IndexError(f"global style token out of range [0, {hi})")
        idx = g.expand(B, n).to(self.device, I32).t().contiguous()   # [n][B]
        out = torch.empty(B, n * d, dtype=F32, device=self.device)
        for j, tab in enumerate(self.gst_tables):
            ops.gather_rows(tab, idx[j], out=out[:, j * d:(j + 1) * d], D=d, M=B)
        return out

    def __call__(self, ids, gfeat=None):
        """ids: device int32 [B, T] codec token ids -> pcm [B, T*upsample] fp32 (tanh output).
        gfeat: optional device fp32 [B, 128] global-style feature per row (global_feature(); None: the configured
        h.global_tokens, as llm2TTS.run passes them).
        Channel-last activations [B][T][C]; every conv on the matrix cores (fo_conv_cl).  On a
        non-default stream the call is one hipGraph replay per (B, T) (captured on first use; the
        ~100 launches of a call otherwise cost more host time than the GPU work)."""
        B, T = ids.shape
        key = (B, T, ops.stream(self.device))   # static buffers per stream: calls on two streams may overlap
        bf = self._graphs.pop(key, None)
        if bf is None:
            if len(self._graphs) >= self.MAX_GRAPHS:   # least recently used (dict order) goes
                okey = next(iter(self._graphs))
                old = self._graphs.pop(okey)
                if old.exec is not None:
                    # its last replay ran on its own stream: wait for that one (a device-wide synchronize would also
                    # wait on -- and, mid-capture, invalidate -- another serving thread's stream)
                    torch.cuda.ExternalStream(okey[2], device=self.device).synchronize()
                    _lib.call("fo_graph_destroy", old.exec)
            bf = self._buffers(B, T)
        self._graphs[key] = bf
        bf.ids.copy_(ids)
        # the graph reads bf.g: per-call global features are copied in, the default restored after them
        if gfeat is not None:
            bf.g.copy_(gfeat)
            bf.g_default = False
        elif not getattr(bf, "g_default", True):
            bf.g.copy_(self.gfeat.view(1, -1).expand(B, -1))
            bf.g_default = True
        st = ops.stream(self.device)
        if not self.use_graphs or st in (0, None):
            self._run(bf)
        else:
            if bf.exec is None:
                _lib.call("fo_graph_begin", st)
                ex = ctypes.c_void_p()
                try:
                    self._run(bf)
                finally:
                    _lib.call("fo_graph_end", st, ctypes.byref(ex))
                bf.exec = ex
            _lib.call("fo_graph_launch", bf.exec, st)
        return bf.out.clone()

    def destroy(self):
        for bf in self._graphs.values():
            if bf.exec is not None:
                _lib.call("fo_graph_destroy", bf.exec)
        self._graphs = {}

    def forward_ncl(self, ids):
        """Channel-major direct-convolution path (VALU kernels of fo_codec.hip); kept as a
        cross-check of the MFMA path."""
        B, T = ids.shape
        dev = self.device
        x = torch.empty(B, 512, T, dtype=F32, device=dev)
        ops.codec_embed(self.codebook, ids.contiguous(), B, T, x)
        w, b = self.conv_pre
        y = torch.empty(B, self.U, T, dtype=F32, device=dev)
        ops.conv1d(x, B, 512, T, w, b, self.U, 7, 1, 3, y)
        x, C, L = y, self.U, T
        g = self.gfeat.view(1, -1).expand(B, -1).contiguous()
        nk = len(self.res[0])
        for i, (w, b, u, k) in enumerate(self.ups):
            Co = C // 2
            Lo = (L - 1) * u - 2 * ((k - u) // 2) + k
            up = torch.empty(B, Co, Lo, dtype=F32, device=dev)
            ops.conv_transpose1d(x, B, C, L, w, b, Co, k, u, (k - u) // 2, up, slope=0.1)
            C, L = Co, Lo
            xs = None
            t1 = torch.empty(B, C, L, dtype=F32, device=dev)
            for kk, convs in self.res[i]:
                yb = up.clone() if xs is not None or nk > 1 else up
                for c1, c2 in convs:
                    w1, b1, d1 = c1
                    if c2 is None:  # ResBlock2: y = conv(leaky(y)) + y
                        ops.conv1d(yb, B, C, L, w1, b1, C, kk, d1, (kk * d1 - d1) // 2, yb, pre_leaky=0.1,
                                   residual=True)
                        continue
                    ops.conv1d(yb, B, C, L, w1, b1, C, kk, d1, (kk * d1 - d1) // 2, t1, pre_leaky=0.1)
                    w2, b2, _ = c2
                    ops.conv1d(t1, B, C, L, w2, b2, C, kk, 1, (kk - 1) // 2, yb, pre_leaky=0.1, residual=True)
                if xs is None:
                    xs = yb
                else:
                    ops.axpy_(xs, yb)
            ops.scale_add_channel_(xs, B, C, L, 1.0 / nk, g if C == g.shape[1] else None)
            x = xs
        w, b = self.conv_post
        out = torch.empty(B, 1, L, dtype=F32, device=dev)
        ops.conv1d(x, B, C, L, w, b, 1, 7, 1, 3, out, pre_leaky=0.1, post_tanh=True)
        return out.view(B, L)


class CodecEncoderEngine:
    """VQVAE.encode (models/decoder/ticodec/vqvae.py:44-57) on fo_codec_enc.hip: Encoder.forward
    (models/decoder/ticodec/models.py:429-522; weight norm removed at load, as Encoder.remove_weight_norm)
    then Quantizer.forward (models.py:639-659).  wav [B, T] fp32 (24 kHz) -> (local ids [B, T', L*G] int32,
    global ids [B, 1, global_code_num] int32), the reference's encode() layout."""

    def __init__(self, src, codec_json, device):
        self.h, self.device = codec_json, torch.device(device)
        self.src = src
        self.p = "codec.encoder."
        rates, ks = codec_json["upsample_rates"], codec_json["upsample_kernel_sizes"]
        self.stages = list(reversed(list(zip(rates, ks))))
        self.rk = list(reversed(codec_json["resblock_kernel_sizes"]))
        self.rd = list(reversed(codec_json["resblock_dilation_sizes"]))
        assert codec_json["resblock"] == "1", "ResBlock1 encoders only (the TiCodec configs use resblock '1')"
        assert 32 * 2 ** len(self.stages) == 512, "Encoder channel ladder must end at conv_post's 512"
        self._w = {}

    def w(self, name):
        if name not in self._w:
            self._w[name] = self.src.get(self.p + name if not name.startswith("codec.") else name).contiguous()
        return self._w[name]

    def _conv(self, x, B, Cin, T, name, stride=1, dil=1, pad=0, pre=None, out=None, residual=False, bias=True):
        wt = self.w(name + ".weight")
        Cout, _, K = wt.shape
        To = (T + 2 * pad - dil * (K - 1) - 1) // stride + 1
        if out is None:
            out = torch.empty(B, Cout, To, dtype=F32, device=self.device)
        ops.conv1d_ex(x, B, Cin, T, wt, self.w(name + ".bias") if bias else None, Cout, K, stride, dil, pad, pre, out,
                      residual)
        return out, Cout, To

    def encoder(self, wav):
        B, T = wav.shape
        x, C, L = self._conv(wav.contiguous(), B, 1, T, "conv_pre", pad=3)
        nk = len(self.rk)
        gfeat = None
        for i, (u, k) in enumerate(self.stages):
            x, C, L = self._conv(x, B, C, L, f"ups.{i}", stride=u, pad=(k - u) // 2, pre=0.1)
            xs = torch.empty_like(x) if nk > 0 else None
            for j in range(nk):
                y = x.clone()
                r = f"resblocks.{i * nk + j}."
                kk = self.rk[j]
                t1 = torch.empty_like(x)
                for m, d in enumerate(self.rd[j]):
                    self._conv(y, B, C, L, r + f"convs1.{m}", dil=d, pad=(kk * d - d) // 2, pre=0.1, out=t1)
                    self._conv(t1, B, C, L, r + f"convs2.{m}", pad=(kk - 1) // 2, pre=0.1, out=y, residual=True)
                if j == 0:
                    xs.copy_(y)
                else:
                    ops.axpy_(xs, y)
                n = f"normalize.{i * nk + j}."
                ops.group_norm(xs, B, C, L, C // 16, self.w(n + "weight"), self.w(n + "bias"), 1e-6,
                               1.0 / nk if j == nk - 1 else 1.0, xs)
            x = xs
            if i == len(self.stages) // 2 - 1:
                gfeat = self.gte(x, B, C, L)
        out, C, L = self._conv(x, B, C, L, "conv_post", pad=1, pre=0.01)   # F.leaky_relu default slope
        return out, gfeat, L

    def gte(self, x, B, C, L):
        _, _, _, k, st = self.h["global_feature_conv"]
        g = "GlobalTokenEncoder."
        for i in (0, 2, 4):
            # leaky 0.1 after each conv = pre-activation of the next consumer (the last one: fo_gte_head)
            x, C, L = self._conv(x, B, C, L, g + f"conv.{i}", stride=st, pad=(k - st) // 2, bias=False,
                                 pre=None if i == 0 else 0.1)
        out = torch.empty(B, C, dtype=F32, device=self.device)
        ops.gte_head(x, B, C, L, self.w(g + "fn.0.weight"), self.w(g + "fn.0.bias"), self.w(g + "fn.2.running_mean"),
                     self.w(g + "fn.2.running_var"), self.w(g + "fn.2.weight"), self.w(g + "fn.2.bias"), 1e-5, out)
        return out

    def encode(self, wav):
        wav = torch.as_tensor(wav)
        if wav.dim() == 3 and wav.shape[-1] == 1:
            wav = wav.squeeze(-1)
        wav = wav.to(self.device, F32).contiguous()
        B = wav.shape[0]
        c, gfeat, L = self.encoder(wav)
        h = self.h
        G, layers = h["n_code_groups"], h["residul_layer"]
        D = 512 // G
        names = ["quantizer_modules", "quantizer_modules2", "quantizer_modules3", "quantizer_modules4"]
        local = torch.empty(B, L, layers * G, dtype=I32, device=self.device)
        res = c   # residual, updated in place
        for li in range(layers):
            for g in range(G):
                cb = self.w(f"codec.quantizer.{names[li]}.{g}.embedding.weight")
                ops.vq_nearest(res, B, 512, L, g * D, D, cb, local, layers * G, li * G + g, residual=True)
        gn = h["global_code_num"]
        gids = torch.empty(B, 1, gn, dtype=I32, device=self.device)
        for g in range(gn):
            cb = self.w(f"codec.quantizer.quantizer_modules_globaltokens.{g}.embedding.weight")
            ops.vq_nearest(gfeat, B, gfeat.shape[1], 1, g * (gfeat.shape[1] // gn), gfeat.shape[1] // gn, cb, gids, gn,
                           g, residual=False)
        return local, gids
