"""DAMSM text-image matching losses (API of miscc/DAMSM_losses.py).

Hot path: ``words_loss`` (DAMSM_losses.py:272-342) and ``sent_loss``
(233-270) run as fused HIP kernels: ONE launch computes func_attention
(25-63), the word-level cosine similarity (17-23) and the log-sum-exp row
similarity for every (image, caption) pair on bf16 MFMA (csrc/damsm.hip), one
launch applies the same-class -inf mask and the bidirectional cross-entropy,
and the backward recomputes the attention in-kernel (no per-sample Python
loop, no ``cap_lens.tolist()`` host sync).

Data parallel (a process group with world > 1): the losses keep the
reference's global-batch semantics (its DataParallel gathers the batch onto
one device, train.py:220-228, 419-435) -- each rank computes its images'
rows against every rank's captions and the blocks are gathered into the
B_global x B_global matrix (eegan_hip.damsm); ``labels`` are the rank's
local match labels (arange(batch_size) from prepare_labels), ``class_ids``
its local ids, and ``batch_size`` the local batch size.

``GlobalAttentionGeneral`` (defined but never called by the reference) runs
as its own HIP kernel (csrc/gag.hip, split-bf16 MFMA, the reference's -inf
mask indexing); ``cosine_similarity``, ``func_attention``, ``sent_similarity``
and ``words_similarity`` are kept for API completeness (also never called on
the training path) as thin tensor expressions.
"""
import torch
import torch.nn as nn

from miscc.config import cfg
from eegan_hip import functional as Fn
from eegan_hip import damsm as G


def cosine_similarity(x1, x2, dim=1, eps=1e-8):
    w12 = torch.sum(x1 * x2, dim)
    return (w12 / (torch.norm(x1, 2, dim) * torch.norm(x2, 2, dim)).clamp(min=eps)).squeeze()


def func_attention(query, context, gamma1):
    B, L = query.size(0), query.size(2)
    ih, iw = context.size(2), context.size(3)
    ctx = context.reshape(B, -1, ih * iw)
    a = torch.softmax(torch.bmm(ctx.transpose(1, 2), query).reshape(B * ih * iw, L), dim=1)
    a = a.reshape(B, ih * iw, L).transpose(1, 2).reshape(B * L, ih * iw)
    a = torch.softmax(a * gamma1, dim=1).reshape(B, L, ih * iw)
    return torch.bmm(ctx, a.transpose(1, 2)), a.reshape(B, -1, ih, iw)


class GlobalAttentionGeneral(nn.Module):
    """word <-> feature-map attention (DAMSM_losses.py:65-132; unused by the reference step).
    Any sourceL (64-source chunks, online softmax); the mask (B, sourceL) bool is applied like the reference's
    ``mask.repeat(queryL, 1)`` (row b*queryL + q reads mask[(b*queryL + q) % B])."""

    def __init__(self, idf, cdf):
        super().__init__()
        self.sm = nn.Softmax(dim=1)
        self.mask = None

    def applyMask(self, mask):
        self.mask = mask

    def forward(self, input, context_key, content_value):
        """-> (weightedContext (B, cdf, ih, iw), attn (B, sourceL, ih, iw)), DAMSM_losses.py:75-132."""
        return Fn.GlobalAttentionFn.apply(input, context_key, content_value, self.mask)


def _masked(sim, class_ids, batch_size):
    cls = G.global_class_ids(class_ids, sim.device)
    if cls is not None:
        n = sim.shape[0]
        m = (cls[None, :] == cls[:n, None]) & ~torch.eye(n, dtype=torch.bool, device=sim.device)
        sim = sim.masked_fill(m, -float('inf'))
    return sim


def sent_similarity(cnn_code, rnn_code, class_ids, batch_size, eps=1e-8):
    return _masked(G.sent_block(cnn_code, rnn_code), class_ids, batch_size)


def sent_loss(cnn_code, rnn_code, labels, class_ids, batch_size, eps=1e-8):
    """(CE(scores, labels), CE(scores^T, labels)); scores = gamma3 * cos, same-class masked."""
    if labels is None:
        return None, None
    sim = G.sent_block(cnn_code, rnn_code)
    losses = Fn.SimCEFn.apply(sim, G.global_class_ids(class_ids, sim.device),
                              G.global_labels(labels, batch_size, sim.device))
    return losses[0], losses[1]


class _AttMaps(object):
    """Lazy ``att_maps`` list of words_loss: element i is attn of (text i, image i),
    shape (1, w_i, 17, 17).  Materialised (with a host read of cap_lens) only on access."""

    def __init__(self, att, cap_lens):
        self._att, self._lens = att, cap_lens

    def __len__(self):
        return self._att.shape[0]

    def __getitem__(self, i):
        w = int(self._lens[i])
        return self._att[i, :w].reshape(1, w, 17, 17)

    def __iter__(self):
        return (self[i] for i in range(len(self)))


def words_similarity(img_features, words_emb, cap_lens, class_ids, batch_size):
    sim, att = G.words_block(img_features, words_emb, cap_lens, True)
    return _masked(sim, class_ids, batch_size), _AttMaps(att, cap_lens)


def words_loss(img_features, words_emb, labels, cap_lens, class_ids, batch_size):
    """Returns (loss0, loss1, att_maps) like DAMSM_losses.py:272-342."""
    sim, att = G.words_block(img_features, words_emb, cap_lens, True)
    maps = _AttMaps(att, cap_lens)
    if labels is None:
        return None, None, maps
    losses = Fn.SimCEFn.apply(sim, G.global_class_ids(class_ids, sim.device),
                              G.global_labels(labels, batch_size, sim.device))
    return losses[0], losses[1], maps
