"""TiCodec vocoder (VQVAE.forward) on the MI355X kernels, batched over sessions.

Reference: models/decoder/ticodec/vqvae.py:37-42 (quantizer.embed + embed_gst + generator),
models/decoder/ticodec/models.py:59-166 (ResBlock1/2), :169-242 (Generator.forward).
"""
import torch

from . import ops
from .ops import F32, I32


class CodecEngine:
    def __init__(self, src, codec_json, device):
        h = self.h = codec_json
        self.device = torch.device(device)
        assert h["residul_layer"] == 1 and h["n_code_groups"] == 1, "single-codebook TiCodec only (the speech decoder emits one id per frame)"
        self.codebook = src.get("codec.quantizer.quantizer_modules.0.embedding.weight", torch.bfloat16)
        gt = h["global_tokens"]
        parts = [src.get(f"codec.quantizer.quantizer_modules_globaltokens.{j}.embedding.weight")[t]
                 for j, t in enumerate(gt)]
        self.gfeat = torch.cat(parts).contiguous()  # [128] (embed_gst, models.py:703-715)
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

    def __call__(self, ids):
        """ids: device int32 [B, T] codec token ids -> pcm [B, T*upsample] fp32 (tanh output).
        Channel-last activations [B][T][C]; every conv on the matrix cores (fo_conv_cl)."""
        B, T = ids.shape
        dev = self.device
        E = self.codebook.shape[1]
        x = torch.empty(B, T, E, dtype=F32, device=dev)
        ops.codec_embed_cl(self.codebook, E, self.codebook.shape[0], ids.contiguous(), B, T, x)
        y = torch.empty(B, T, self.U, dtype=F32, device=dev)
        ops.conv_cl(x, B, E, T, self.p_pre, 1, 3, y)
        x, C, L = y, self.U, T
        g = self.gfeat.view(1, -1).expand(B, -1).contiguous()
        nk = len(self.res[0])
        for i, (w, b, u, k) in enumerate(self.ups):
            Co = C // 2
            Lo = (L - 1) * u - 2 * ((k - u) // 2) + k
            up = torch.empty(B, Lo, Co, dtype=F32, device=dev)
            for r, pc, pad_r in self.p_ups[i]:  # leaky -> ConvTranspose1d as u polyphase convs
                Tq = (Lo - r + u - 1) // u
                ops.conv_cl(x, B, C, L, pc, 1, pad_r, up, Tq=Tq, ostride=u, ooff=r, Tout_total=Lo, pre_leaky=0.1)
            C, L = Co, Lo
            xs = None
            t1 = torch.empty(B, L, C, dtype=F32, device=dev)
            for kk, convs in self.p_res[i]:
                yb = up.clone() if xs is not None or nk > 1 else up
                for p1, d1, p2 in convs:
                    if p2 is None:  # ResBlock2: y = conv(leaky(y)) + y
                        ops.conv_cl(yb, B, C, L, p1, d1, (kk * d1 - d1) // 2, yb, pre_leaky=0.1, residual=True)
                        continue
                    ops.conv_cl(yb, B, C, L, p1, d1, (kk * d1 - d1) // 2, t1, pre_leaky=0.1)
                    ops.conv_cl(t1, B, C, L, p2, 1, (kk - 1) // 2, yb, pre_leaky=0.1, residual=True)
                if xs is None:
                    xs = yb
                else:
                    ops.axpy_(xs, yb)
            ops.scale_add_cl(xs, B, L, C, 1.0 / nk, g if C == g.shape[1] else None)
            x = xs
        w, b = self.conv_post
        out = torch.empty(B, L, dtype=F32, device=dev)
        ops.conv_post_cl(x, B, L, C, w, b, w.shape[-1], (w.shape[-1] - 1) // 2, 0.1, out)
        return out

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
