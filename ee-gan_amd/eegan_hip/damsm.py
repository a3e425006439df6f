"""Global-batch DAMSM similarity blocks for data-parallel ranks.

Under the reference's single-process nn.DataParallel the DAMSM losses see the
whole gathered batch: region features / codes of every fake image against
every caption, same-class masks over the global class ids
(train.py:419-435, miscc/DAMSM_losses.py:233-342).  One process per GPU
reproduces that without gathering image features: each rank computes the
rows of ITS images against ALL ranks' captions (captions, lengths, class ids
and labels are all-gathered; they carry no gradient in the training step),
then the B_local x B_global similarity blocks are all-gathered into the
B_global x B_global matrix (differentiable: backward is the rank's rows of the
summed gradient), and the masked bidirectional cross-entropy runs on it.
Every rank then holds the same global loss; its image-side gradient arrives
W-fold through the gather's backward, which the data-parallel gradient
averaging (/W) turns back into exactly the reference's gradient.

At world 1 (or without a process group) every helper is the identity and the
blocks are the plain B x B matrices.
"""
import torch

from . import dist as D
from . import functional as Fn


def _dev_long(x, device):
    if x is None:
        return None
    return torch.as_tensor(x).to(device=device, dtype=torch.long, non_blocking=True).reshape(-1).contiguous()


def gather_texts(t):
    """Captions' embeddings / lengths / ids of all ranks (identity at world 1)."""
    if t is None or not D.collective():
        return t
    return D.all_gather(t, differentiable=t.requires_grad)


def global_labels(labels, b_local, device):
    """match labels of the gathered batch: rank r's label l becomes r*B_local + l."""
    if labels is None:
        return None
    lab = _dev_long(labels, device)
    if not D.collective():
        return lab
    return D.all_gather(lab + D.rank() * b_local, differentiable=False)


def global_class_ids(class_ids, device):
    ids = _dev_long(class_ids, device)
    if ids is None or not D.collective():
        return ids
    return D.all_gather(ids, differentiable=False)


WORDS_PAD = 32   # csrc/damsm.hip NW: the widest caption the words kernel takes


def words_block(regions, words_emb, cap_lens, want_att=False):
    """(sim B_global x B_global, att maps of this rank's matching pairs)."""
    dev = regions.device
    lens = _dev_long(cap_lens, dev)
    off = 0
    if D.collective():
        off = D.rank() * regions.shape[0]
        # every rank's words padded to the kernel's 32-word width before the
        # gather: a rank's T is ITS batch's longest caption, so the ranks'
        # tensors would differ in size; the padding is zeros past each
        # caption's length -- what the reference's pad_packed_sequence gives
        # the global batch -- and the kernel masks those positions anyway
        T = words_emb.shape[2]
        if T < WORDS_PAD:
            words_emb = torch.nn.functional.pad(words_emb, (0, WORDS_PAD - T))
        words_emb = gather_texts(words_emb)
        lens = gather_texts(lens)
    sim, att = Fn.WordsSimFn.apply(regions, words_emb, lens, want_att, off)
    return D.all_gather(sim), att


def sent_block(cnn_code, rnn_code):
    """gamma3 * cos over (all images) x (all captions), rows computed locally."""
    return D.all_gather(Fn.SentSimFn.apply(cnn_code, gather_texts(rnn_code)))
