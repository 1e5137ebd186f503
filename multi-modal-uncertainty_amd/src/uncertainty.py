"""K-member deep ensemble x T-pass MC-dropout evaluation of MMBT, NLL and ECE.

North-star feature (absent from the reference code).
The K members share the architecture but not the weights; their 12 encoder layers
run as ONE batched launch per op: every GEMM is batched over members (weight
stride = one member's matrix), attention is weight-free so all K*T*B sequences
go in one launch, and LayerNorm uses member-strided affine params
(mmu_layernorm_fwd group_rows).  MC-dropout replicates each batch T times inside
a member; dropout masks differ per row because the dropout counters include the
row index.  ResNet-152 (MIOpen) and the token embedding run per member.

Metrics (mmu_uncertainty / mmu_ece_bins):
  p_bar = mean over the K*T rows of softmax(logits)    (notebooks/food101_robustness.py:25-36)
  NLL   = -mean log p_bar[y]      (== reference CrossEntropyLoss at K = T = 1, src/mmbt.py:243)
  ECE   = sum_b (n_b/N) |acc_b - conf_b| over 15 equal-width bins of max p_bar (build-defined)
"""
import numpy as np
import torch

from . import kernels as K
from .mmbt import LN_EPS, _mix, _seed

bf16 = torch.bfloat16
HID, FFN = 768, 3072


class EnsembleMMBT:
    """Stacked view of K MultimodalBertClf members (all on one device, eval mode)."""

    KEYS = ("wqkv16", "bqkv", "wo16", "bo", "ln1w", "ln1b", "w116", "b1", "w216", "b2", "ln2w", "ln2b")

    def __init__(self, members):
        self.members = list(members)
        self.K = len(self.members)
        for m in self.members:
            m.eval()
            m.enc._prepare()
        n_layers = len(self.members[0].enc._lw)
        self.layers = []
        for i in range(n_layers):
            self.layers.append({k: torch.stack([getattr(m.enc._lw[i], k) for m in self.members]).contiguous()
                                for k in self.KEYS})
        enc0 = self.members[0].enc
        self.pool_w = torch.stack([m.enc.pooler.dense.weight.detach() for m in self.members])
        self.pool_b = torch.stack([m.enc.pooler.dense.bias.detach() for m in self.members])
        self.clf_w = torch.stack([m.clf.weight.detach() for m in self.members])
        self.clf_b = torch.stack([m.clf.bias.detach() for m in self.members])
        self.hidden_dropout, self.attn_dropout = enc0.hidden_dropout, enc0.attn_dropout

    def _layer(self, lw, X, R, km, nb, L, p_attn, p_hid, seeds, res_ln=None, out32=False):
        """X bf16 [K*M, 768] + its f32 residual -> (Y, S2, mean2, rstd2, Y32): src/encoder.py
        layer_forward batched over the members (the same f32 hidden stream: R is the embeddings'
        f32 rows, or the previous layer's S2 whose LayerNorm the epilogue recomputes from
        res_ln = (mean, rstd, gamma [K, 768], beta [K, 768]))."""
        Km, M = self.K, nb * L
        dev = X.device
        f32 = torch.float32
        qkv = torch.empty(Km * M, 3 * HID, dtype=bf16, device=dev)
        K.gemm(X, HID, True, lw["wqkv16"], HID, True, qkv, 3 * HID, M, 3 * HID, HID, batch=Km, sA=M * HID,
               sB=3 * HID * HID, sC=M * 3 * HID, epi=K.epilogue(K.EPI_STORE, bias=lw["bqkv"], bias_bstride=3 * HID))
        O = torch.empty(Km * M, HID, dtype=bf16, device=dev)
        lse = torch.empty(Km * nb * 12, L, dtype=torch.float32, device=dev)
        K.attention_fwd(qkv, km, O, lse, Km * nb, L, 12, p_attn, seeds[0])
        S1 = torch.empty(Km * M, HID, dtype=f32, device=dev)
        K.gemm(O, HID, True, lw["wo16"], HID, True, S1, HID, M, HID, HID, batch=Km, sA=M * HID, sB=HID * HID,
               sC=M * HID, epi=K.epilogue(K.EPI_BIAS_DROP_RES, bias=lw["bo"], bias_bstride=HID, residual=R,
                                          res_bstride=M * HID, drop_p=p_hid, seed=seeds[1], res_ln=res_ln,
                                          res_ln_bstride=HID))
        del R
        A = torch.empty_like(O)
        mean1 = torch.empty(Km * M, dtype=f32, device=dev)
        rstd1 = torch.empty_like(mean1)
        K.layernorm_fwd_f32(S1, lw["ln1w"], lw["ln1b"], A, None, mean1, rstd1, eps=LN_EPS, group_rows=M,
                            param_stride=HID)
        Hh = torch.empty(Km * M, FFN, dtype=bf16, device=dev)
        K.gemm(A, HID, True, lw["w116"], HID, True, Hh, FFN, M, FFN, HID, batch=Km, sA=M * HID, sB=FFN * HID,
               sC=M * FFN, epi=K.epilogue(K.EPI_BIAS_GELU, bias=lw["b1"], bias_bstride=FFN))
        del A
        S2 = torch.empty(Km * M, HID, dtype=f32, device=dev)
        K.gemm(Hh, FFN, True, lw["w216"], FFN, True, S2, HID, M, HID, FFN, batch=Km, sA=M * FFN, sB=HID * FFN,
               sC=M * HID, epi=K.epilogue(K.EPI_BIAS_DROP_RES, bias=lw["b2"], bias_bstride=HID, residual=S1,
                                          res_bstride=M * HID, drop_p=p_hid, seed=seeds[2],
                                          res_ln=(mean1, rstd1, lw["ln1w"], lw["ln1b"]), res_ln_bstride=HID))
        del S1, Hh
        Y = torch.empty_like(O)
        Y32 = torch.empty_like(S2) if out32 else None
        mean2 = torch.empty(Km * M, dtype=f32, device=dev)
        rstd2 = torch.empty_like(mean2)
        K.layernorm_fwd_f32(S2, lw["ln2w"], lw["ln2b"], Y, Y32, mean2, rstd2, eps=LN_EPS, group_rows=M,
                            param_stride=HID)
        return Y, S2, mean2, rstd2, Y32

    @torch.no_grad()
    def logits(self, txt, mask, segment, img, mc_samples=1, mc_dropout=None):
        """-> [K, T, B, n_classes] f32.  mc_dropout defaults to mc_samples > 1."""
        mc = (mc_samples > 1) if mc_dropout is None else mc_dropout
        T_mc = int(mc_samples)
        B, Tt = txt.shape
        enc0 = self.members[0].enc
        S = enc0.n_img + 2 + Tt
        nb = T_mc * B
        M = nb * S
        dev = img.device
        X = torch.empty(self.K * M, HID, dtype=bf16, device=dev)
        X32 = torch.empty(self.K * M, HID, dtype=torch.float32, device=dev)
        km = torch.empty(self.K * nb, S, dtype=torch.float32, device=dev)
        p_txt = self.hidden_dropout if mc else 0.0
        idx = torch.arange(S, device=dev).repeat(T_mc, 1)  # T_mc copies of the identity gather
        txt, segment, mask = (t.contiguous().long() for t in (txt, segment, mask))
        for k, m in enumerate(self.members):
            e = m.enc
            proj = e.img_embeddings.project(e._image_feats(img)).contiguous()
            et = e.txt_embeddings
            K.embed_fwd(txt, segment, mask, proj, et.word_embeddings.weight, et.position_embeddings.weight,
                        et.token_type_embeddings.weight, et.LayerNorm.weight, et.LayerNorm.bias, LN_EPS, e.cls_id,
                        e.sep_id, idx, T_mc, B, Tt, e.n_img, S, X[k * M:(k + 1) * M], km[k * nb:(k + 1) * nb],
                        drop_txt=p_txt, drop_img=0.0, seed=_seed() if mc else 0, X32=X32[k * M:(k + 1) * M])
        p_attn, p_hid = (self.attn_dropout, self.hidden_dropout) if mc else (0.0, 0.0)
        base = _seed() if mc else 0
        R, rln, n = X32, None, len(self.layers)
        del X32
        for i, lw in enumerate(self.layers):
            X, R, mu, rs, Y32 = self._layer(lw, X, R, km, nb, S, p_attn, p_hid,
                                            (_mix(base, 3 * i), _mix(base, 3 * i + 1), _mix(base, 3 * i + 2)),
                                            rln, out32=i == n - 1)
            rln = (mu, rs, lw["ln2w"], lw["ln2b"])
        h0 = Y32.view(self.K, nb, S, HID)[:, :, 0]                             # [K, nb, 768] f32
        pooled = torch.tanh(torch.baddbmm(self.pool_b.unsqueeze(1), h0, self.pool_w.transpose(1, 2)))
        out = torch.baddbmm(self.clf_b.unsqueeze(1), pooled, self.clf_w.transpose(1, 2))
        return out.view(self.K, T_mc, B, -1)


class UncertaintyMeter:
    """Accumulates NLL / ECE bins / accuracy over batches with the HIP reduction kernels."""

    def __init__(self, n_bins=15):
        self.n_bins = n_bins
        self.bins = None
        self.nll_sum = 0.0
        self.correct = 0.0
        self.count = 0

    def update(self, logits, y):
        """logits [S, R, C] (R = members x passes), y [S]."""
        S, R, C = logits.shape
        dev = logits.device
        p_bar = torch.empty(S, C, dtype=torch.float32, device=dev)
        nll, conf, cor = (torch.empty(S, dtype=torch.float32, device=dev) for _ in range(3))
        K.uncertainty(logits.float().contiguous(), y.long().contiguous(), p_bar, nll, conf, cor)
        bins = torch.empty(3 * self.n_bins, dtype=torch.float32, device=dev)
        K.ece_bins(conf, cor, self.n_bins, bins)
        b = bins.double().cpu().numpy()
        self.bins = b if self.bins is None else self.bins + b
        self.nll_sum += float(nll.double().sum())
        self.correct += float(cor.double().sum())
        self.count += S
        return p_bar

    def result(self):
        bb = self.bins.reshape(self.n_bins, 3)
        ece = float(np.abs(bb[:, 2] - bb[:, 1]).sum() / max(self.count, 1))
        return {"nll": self.nll_sum / max(self.count, 1), "ece": ece, "acc": self.correct / max(self.count, 1),
                "n": self.count}
