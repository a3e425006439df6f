"""The EE-GAN inner G/D training step on MI355X (mirror of train.py:90-103,
148-206, 252-263, 336-502).

Method names, arguments and the order of operations follow the reference
Trainer so the step reads like train.py; the arithmetic of every loss runs in
HIP kernels (hinge means, BCE-with-logits, the MA gradient penalty, masked
bidirectional CE of the DAMSM losses), the optimizers are flat fused Adams,
and nothing in the step reads device memory on the host (no .item(), no
cap_lens.tolist()).  Scalar loss combinations stay torch expressions on
0-d tensors.
"""
import collections
import contextlib
import os
import sys

import torch

from . import functional as Fn
from . import dist as D
from . import damsm as G
from .optim import FlatAdam
from .tensor import new_stream


def prepare_labels(batch_size, device):
    """train.py:90-97."""
    real = torch.ones(batch_size, device=device)
    fake = torch.zeros(batch_size, device=device)
    match = torch.arange(batch_size, device=device)
    return real, fake, match


def prepare_class_labels(batch_size, class_num, class_ids, device):
    """train.py:99-103 on the device: labels[i][(id_i - 1) mod class_num] = 1 (bit-exact)."""
    lab, _ = Fn.class_onehot(class_ids, batch_size, class_num, device)
    return lab


# EEGAN_LANE_PRIO: 1 the largest D's lane at the highest stream priority, the
# others default; 2 the others at the lowest priority too; 0 all default
LANE_PRIO = int(os.environ.get('EEGAN_LANE_PRIO', '1'))
# EEGAN_G_EARLY=0: g_update's passes through the three D's wait for all of d_update.
G_EARLY = os.environ.get('EEGAN_G_EARLY', '1') != '0'
# EEGAN_DAMSM_EARLY=0: the DAMSM branch runs inside g_update, after d_update (A/B switch).
DAMSM_EARLY = os.environ.get('EEGAN_DAMSM_EARLY', '1') != '0'
# EEGAN_DAMSM_GRAD_EARLY=0: the DAMSM branch's backward waits for g_update's backward (A/B switch).
DAMSM_GRAD_EARLY = os.environ.get('EEGAN_DAMSM_GRAD_EARLY', '1') != '0'
# EEGAN_GTERM_GRAD_EARLY=n: g_update's term through D i (i < n; n = -1: every D) is
# differentiated w.r.t. its fake image on D i's lane right after the term's
# forward (g_loss is linear in the per-D terms, train.py:477-493), so the
# smaller D's input-gradient passes run while the largest D's update still
# holds the critical lane instead of beside g_update's backward; 0 = off (A/B switch).
GTERM_GRAD_EARLY = int(os.environ.get('EEGAN_GTERM_GRAD_EARLY', '-1'))   # -1: +1.9 % (profiles/r03_gterm_early.txt)
# the discriminator lanes are issued largest (critical) first and the DAMSM lane after them: the
# first packets of the critical lane then do not queue behind the others' (C2: 678 vs 656 img/s,
# tools/gpu_env_ab.sh); EEGAN_LANE_ORDER=fwd: D64, D128, D256 after the DAMSM lane
LANE_ORDER = os.environ.get('EEGAN_LANE_ORDER', 'rev')
# False: the generator's stage 2-3 Cum_Block / image branches stay on the main
# stream (models.Gen.forward_branched puts them on D64's idle lane; module
# constant for A/B: tools/ab_inproc.py "py:eegan_hip.trainer.GEN_SIDE=False")
GEN_SIDE = True
# True (N > 1 with stream lanes): the largest discriminator's and the generator's
# gradient buckets are all-reduced on communication lanes of their own (streams
# forked from the step's origin stream, own RCCL communicators), so their
# backward kernels do not queue behind the reductions; each optimizer's step
# waits for its lane (FlatAdam.comm_stream).  Module constant for A/B.
COMM_LANES = True
# Lanes whose convs are planned for throughput (eegan_conv_desc.plan = 1: larger
# tiles, no split-K partials or reduce launches) -- lanes that run beside the
# critical chain, where a conv's latency matters less than the CU time it takes
# from the critical lane.  Indices of _side_streams: 0..nD-1 the discriminators'
# lanes (0 also carries the generator's stage 2-3 branch), nD the DAMSM lane.
# EEGAN_TP_LANES: comma-separated indices ('' = none).
TP_LANES = tuple(int(v) for v in os.environ.get('EEGAN_TP_LANES', '').split(',') if v.strip())
# Measured alternatives kept as module constants (A/B: tools/ab_inproc.py
# "py:eegan_hip.trainer.NAME=value"; DESIGN.md §3, round 5, all behind the default):
# DREAL_EARLY -- discriminators whose real-image share of d_loss (the real and
# mismatch heads, train.py:338-341 / 357-364: they read the real images, the text
# embeddings and D's weights as they are at the step's start, nothing the generator
# makes) is computed and back-propagated right after the text encoder, beside the
# generator's forward, d_update then adding only the fake-image share before the
# first Adam step (d_loss is a sum over the heads: the same gradient in another
# accumulation order); DREAL_LANE -- on the D's own lane ('own') or the DAMSM lane
# ('damsm', joined by the origin stream before d_update forks);
# LANE_GATE -- {i: (j, phase)}: D i's lane forked from the origin stream only once
# D j's lane has issued `phase` (one of LANE_PHASES).
DREAL_EARLY = ()
DREAL_LANE = 'own'
LANE_PHASES = ('loss', 'adam', 'gp', 'gpadam', 'gterm')
LANE_GATE = {}

# a g_update term already differentiated w.r.t. its fake image on its lane
# (GTERM_GRAD_EARLY): its value, the image alias and the gradient there
EarlyTerm = collections.namedtuple('EarlyTerm', 'value alias grad')


def _backward_roots(terms):
    """(roots, grads) for g_update's backward from per-D terms: a plain term
    is a root with gradient 1, an EarlyTerm enters at its image alias."""
    roots, grads = [], []
    for t in terms:
        if isinstance(t, EarlyTerm):
            roots.append(t.alias)
            grads.append(t.grad)
        else:
            roots.append(t)
            grads.append(None)
    return roots, grads


def _term_value(t):
    return t.value if isinstance(t, EarlyTerm) else t


class Trainer(object):
    def __init__(self, netG, attr_enhance, netsD, image_encoder, text_encoder, batch_size, disc_class=True,
                 class_nums=200, class_coe=10.0, sim_coe=0.05, device='cuda', max_attr_nums=3, damsm_global=True,
                 streams=None):
        self.netG, self.attr_enhance, self.netsD = netG, attr_enhance, netsD
        self.image_encoder, self.text_encoder = image_encoder, text_encoder
        self.batch_size = batch_size
        self.disc_class, self.class_nums = disc_class, class_nums
        self.d_class_coe = self.g_class_coe = class_coe
        self.DAMSM_coe = sim_coe
        self.device = device
        self.max_attr_nums = max_attr_nums
        self.damsm_global = damsm_global
        self.optimizerG, self.optimizerDs = self.load_optimizers(netG, netsD, attr_enhance)
        self.records = {}
        # the three discriminators share no parameters, so their d_update
        # sequences (and, in g_update, their forward/backward on the fake images
        # beside the DAMSM image encoder) run on separate HIP streams: the small
        # 64/128-px launches fill the GPU next to the 256-px ones.  Every phase
        # forks from and joins back into the caller's stream, so a captured step
        # graph sees the same dependencies.
        if streams is None:
            streams = os.environ.get('EEGAN_STREAMS', '1') != '0'
        self.use_streams = bool(streams) and torch.cuda.is_available() and torch.device(device).type == 'cuda'
        self._streams = None

    def _side_streams(self, n, fork=True):
        if not self.use_streams:
            return [None] * n
        # lanes 4 / 5 carry the communication lanes' RCCL communicators (_comm_lanes): a
        # compute lane bound to the same communicator would issue on it from a second stream
        assert n <= 4, 'at most 4 compute lanes (communicators 4 and 5 are the comm lanes)'
        if self._streams is None or len(self._streams) < n:
            # the last discriminator's lane (the largest D: the step's critical
            # path through d_update and g_update) at high priority, the others
            # filling around it (EEGAN_LANE_PRIO=0: all default)
            hi = len(self.netsD) - 1 if LANE_PRIO else -1
            lo = -1 if LANE_PRIO == 2 else 0
            self._streams = [new_stream(self.device, 1 if i == hi else lo) for i in range(n)]
            for i, st in enumerate(self._streams):
                D.bind_stream(st, i)   # one RCCL communicator per stream lane
        for i, st in enumerate(self._streams):   # planner objective per lane (TP_LANES)
            if i in TP_LANES:
                Fn.STREAM_PLAN[st.cuda_stream] = 1
            else:
                Fn.STREAM_PLAN.pop(st.cuda_stream, None)
        if fork:
            main = torch.cuda.current_stream()
            for s in self._streams[:n]:
                s.wait_stream(main)
        return self._streams[:n]

    def _comm_lanes(self):
        """The communication lanes (N > 1): created once, bound to communicators
        5 and 6 (eegan_hip.dist lanes 4 / 5) and handed to the optimizers."""
        if not (COMM_LANES and self.use_streams and D.collective()):
            return []
        if getattr(self, '_comm', None) is None:
            self._comm = [new_stream(self.device, 0) for _ in range(2)]
            for i, st in enumerate(self._comm):
                D.bind_stream(st, 4 + i)
            self.optimizerDs[-1].comm_stream = self._comm[0]
            self.optimizerG.comm_stream = self._comm[1]
        return self._comm

    @staticmethod
    def _on(stream):
        return torch.cuda.stream(stream) if stream is not None else contextlib.nullcontext()

    @staticmethod
    def _join(streams):
        main = torch.cuda.current_stream()
        for s in streams:
            if s is not None:
                main.wait_stream(s)

    @staticmethod
    def load_optimizers(netG, netDs, attr_enhance):
        """train.py:252-263: Adam(betas=(0, 0.9)), G+ATTR lr 1e-4, each D lr 4e-4."""
        pg = torch.distributed.group.WORLD if D.is_on() else None
        EG = [p for p in list(netG.parameters()) + list(attr_enhance.parameters()) if p.requires_grad]
        optG = FlatAdam(EG, lr=0.0001, betas=(0.0, 0.9), process_group=pg)
        optDs = [FlatAdam([p for p in d.parameters() if p.requires_grad], lr=0.0004, betas=(0.0, 0.9),
                          process_group=pg) for d in netDs]
        return optG, optDs

    # ------------------------------------------------------------ losses --
    # D has no batch-coupled layer, so the real and fake passes of d_loss (and
    # the real / mismatch / fake heads) run as ONE batch: the same per-sample
    # outputs and summed gradients as train.py's separate calls, half the
    # trunk launches and twice the work per launch (EEGAN_DBATCH=0: separate)
    DBATCH = os.environ.get('EEGAN_DBATCH', '1') != '0'

    @staticmethod
    def _d_heads_batched(imgs, fake_imgs, sent_emb, wrong_sent_emb, netD):
        B = imgs.shape[0]
        feat = netD(Fn.BatchCatFn.apply(imgs, fake_imgs.detach()))
        heads = Fn.HeadsGatherFn.apply(feat, B)  # [real; real; fake]
        cond = torch.cat([sent_emb.reshape(B, -1), wrong_sent_emb.reshape(B, -1), sent_emb.reshape(B, -1)], 0)
        return netD.module.COND_DNET(heads, cond), B

    @staticmethod
    def d_loss(imgs, fake_imgs, sent_emb, wrong_sent_emb, netD):
        """train.py:336-353."""
        if Trainer.DBATCH:
            out, B = Trainer._d_heads_batched(imgs, fake_imgs, sent_emb, wrong_sent_emb, netD)
            return Fn.DoutReduce3Fn.apply(out, B, (0, 1, 1))  # real, fake, mismatch
        real_features = netD(imgs)
        real_out = netD.module.COND_DNET(real_features, sent_emb)
        errD_real = Fn.DoutReduceFn.apply(real_out, 0)
        unpair_out = netD.module.COND_DNET(real_features, wrong_sent_emb)
        errD_mismatch = Fn.DoutReduceFn.apply(unpair_out, 1)
        fake_features = netD(fake_imgs.detach())
        fake_out = netD.module.COND_DNET(fake_features, sent_emb)
        errD_fake = Fn.DoutReduceFn.apply(fake_out, 1)
        return errD_real, errD_fake, errD_mismatch

    @staticmethod
    def d_loss_class(imgs, fake_imgs, sent_emb, unpair_sent_emb, class_labels, netD):
        """train.py:355-376."""
        if Trainer.DBATCH:
            (sent_out, class_out), B = Trainer._d_heads_batched(imgs, fake_imgs, sent_emb, unpair_sent_emb, netD)
            return (*Fn.DoutReduce3Fn.apply(sent_out, B, (0, 1, 1)),  # real, fake, mismatch
                    *Fn.BceLogits3Fn.apply(class_out, class_labels))
        real_feature = netD(imgs)
        real_sent_out, real_class_out = netD.module.COND_DNET(real_feature, sent_emb)
        errD_real = Fn.DoutReduceFn.apply(real_sent_out, 0)
        errD_real_class = Fn.BceLogitsFn.apply(real_class_out, class_labels)
        unpair_sent_out, unpair_class_out = netD.module.COND_DNET(real_feature, unpair_sent_emb)
        errD_mismatch = Fn.DoutReduceFn.apply(unpair_sent_out, 1)
        errD_mismatch_class = Fn.BceLogitsFn.apply(unpair_class_out, class_labels)
        fake_features = netD(fake_imgs.detach())
        fake_sent_out, fake_class_out = netD.module.COND_DNET(fake_features, sent_emb)
        errD_fake = Fn.DoutReduceFn.apply(fake_sent_out, 1)
        errD_fake_class = Fn.BceLogitsFn.apply(fake_class_out, class_labels)
        return errD_real, errD_fake, errD_mismatch, errD_real_class, errD_fake_class, errD_mismatch_class

    @staticmethod
    def d_loss_real(imgs, sent_emb, wrong_sent_emb, class_labels, netD, disc_class):
        """The real-image heads of d_loss / d_loss_class (train.py:338-341,
        357-364): (errD_real, errD_mismatch[, errD_real_class, errD_mismatch_class])
        from ONE pass of D over the real images."""
        B = imgs.shape[0]
        feat = netD(imgs)
        heads = Fn.BatchCatFn.apply(feat, feat)   # [real; real]: sentence / mismatched sentence
        cond = torch.cat([sent_emb.reshape(B, -1), wrong_sent_emb.reshape(B, -1)], 0)
        out = netD.module.COND_DNET(heads, cond)
        if disc_class:
            s, c = out
            return (Fn.DoutReduceFn.apply(s[:B], 0), Fn.DoutReduceFn.apply(s[B:], 1),
                    Fn.BceLogitsFn.apply(c[:B], class_labels), Fn.BceLogitsFn.apply(c[B:], class_labels))
        return Fn.DoutReduceFn.apply(out[:B], 0), Fn.DoutReduceFn.apply(out[B:], 1)

    @staticmethod
    def d_loss_fake(fake_imgs, sent_emb, class_labels, netD, disc_class):
        """The fake-image head of d_loss / d_loss_class (train.py:342-344,
        365-368): (errD_fake[, errD_fake_class])."""
        out = netD.module.COND_DNET(netD(fake_imgs.detach()), sent_emb)
        if disc_class:
            return Fn.DoutReduceFn.apply(out[0], 1), Fn.BceLogitsFn.apply(out[1], class_labels)
        return (Fn.DoutReduceFn.apply(out, 1),)

    def d_real_early(self, i, imgs, sent_emb, unpair_sent_emb, class_labels):
        """D i's real-image share of d_loss, differentiated into its zeroed
        gradient on the current stream (DREAL_EARLY); returns the head values."""
        disc_class = self.disc_class and i == 2
        optD = self.optimizerDs[i]
        Fn.stamp('D%d real start' % i)
        vals = self.d_loss_real(imgs[i], sent_emb, unpair_sent_emb, class_labels, self.netsD[i], disc_class)
        part = vals[0] + vals[1] / 2.0
        if disc_class:
            part = part + (vals[2] + vals[3]) / 3.0 * self.d_class_coe
        optD.zero_grad()
        part.backward(inputs=optD.params)
        Fn.stamp('D%d real forward + backward' % i)
        return tuple(v.detach() for v in vals)

    @staticmethod
    def MA_gradient_penalty(imgs, sent_emb, netD, disc_class):
        """train.py:378-402: 2 * mean(||d D(x,s) / d(x,s)||^6), double backward."""
        interpolated = imgs.detach().requires_grad_()
        sent_inter = sent_emb.detach().requires_grad_()
        features = netD(interpolated)
        if disc_class:
            out, _ = netD.module.COND_DNET(features, sent_inter)
        else:
            out = netD.module.COND_DNET(features, sent_inter)
        # the first backward's act' masks read their activations detached (piecewise
        # constant: no gradient flows into them), so the second backward never walks
        # the forward graph with zero-filled gradients (functional._mask_src)
        with Fn.detached_mask_sources(Fn.GP_DETACH_MASKS):
            grads = torch.autograd.grad(outputs=out, inputs=(interpolated, sent_inter),
                                        grad_outputs=torch.ones_like(out), retain_graph=True, create_graph=True,
                                        only_inputs=True)
        return Fn.GradPenaltyFn.apply(grads[0], grads[1])

    @staticmethod
    def g_loss_class(fake_imgs, sent_emb, class_labels, netD):
        features = netD(fake_imgs)
        fake_sent, fake_class = netD.module.COND_DNET(features, sent_emb)
        return Fn.DoutReduceFn.apply(fake_sent, 2), Fn.BceLogitsFn.apply(fake_class, class_labels)

    @staticmethod
    def g_loss(fake_imgs, sent_emb, netD):
        features = netD(fake_imgs)
        return Fn.DoutReduceFn.apply(netD.module.COND_DNET(features, sent_emb), 2)

    def DAMSM_loss(self, fake_imgs, sent_emb, words_embs, attrs_emb, class_ids, batch_size, match_labels, cap_lens,
                   image_encoder):
        """train.py:419-435 over the GLOBAL batch when data-parallel: this rank's
        image rows against every rank's captions, the similarity blocks gathered
        (eegan_hip.damsm; damsm_global=False keeps the losses per rank)."""
        region_features, cnn_code = image_encoder(fake_imgs)
        if Fn.STAMPS is not None:   # diagnostics: when the losses' gradient reaches the image encoder
            region_features.register_hook(lambda g: (Fn.stamp('dregions ready'), g)[1])
        dev = cnn_code.device
        if self.damsm_global:
            cls = G.global_class_ids(class_ids, dev)
            lab = G.global_labels(match_labels, batch_size, dev)
            s_sim = G.sent_block(cnn_code, sent_emb)
            w_sim, _ = G.words_block(region_features, words_embs, cap_lens)
            a_sim = G.sent_block(cnn_code, attrs_emb)
        else:
            cls = G._dev_long(class_ids, dev)
            lab = G._dev_long(match_labels, dev)
            s_sim = Fn.SentSimFn.apply(cnn_code, sent_emb)
            w_sim, _ = Fn.WordsSimFn.apply(region_features, words_embs, G._dev_long(cap_lens, dev), False)
            a_sim = Fn.SentSimFn.apply(cnn_code, attrs_emb)
        s = Fn.SimCEFn.apply(s_sim, cls, lab)
        w = Fn.SimCEFn.apply(w_sim, cls, lab)
        a = Fn.SimCEFn.apply(a_sim, cls, lab)
        lam = 1.0
        return (w[0] + w[1]) * lam, (s[0] + s[1]) * lam, (a[0] + a[1]) * lam

    # ----------------------------------------------------------- updates --
    def d_update(self, imgs, fake_imgs, sent_emb, unpair_sent_emb, class_labels, iter_rec=False, g_early=None,
                 before_join=None, real=None):
        """train.py:437-469: per D a hinge(+class) step, then a GP step (each D
        on its own stream).  `g_early` (a list): also run g_update's generator
        loss term through each D right after that D's update, into the list.
        `real`: {D index: real-image head values} of d_real_early."""
        nD = len(self.netsD)
        streams = self._side_streams(nD)
        g_terms = [None] * nD
        order = range(nD)
        if LANE_ORDER == 'rev':
            order = reversed(order)
        order = list(order)
        gates = {i: g for i, g in LANE_GATE.items() if i < nD and g[0] < nD and g[0] != i} if self.use_streams else {}
        gens, pos = {}, {}

        def lane(i):
            Fn.stamp('D%d start' % i)
            yield from self._d_update_one(i, imgs, fake_imgs, sent_emb, unpair_sent_emb, class_labels, iter_rec,
                                          real=(real or {}).get(i))
            if g_early is not None:
                # g_update's pass through this D (train.py:477-489) reads only this D's
                # final parameters and the fake images: it runs on the lane as soon as
                # the update is done, while the larger D's update still runs
                g_terms[i] = self._g_term(i, fake_imgs, sent_emb, class_labels, iter_rec)
            yield 'gterm'

        def advance(i, until=None):
            """Issue lane i's phases up to and including `until` (None: all)."""
            if i not in gens:
                gens[i], pos[i] = lane(i), -1
            if until is not None and pos[i] >= LANE_PHASES.index(until):
                return
            with self._on(streams[i]):
                for ph in gens[i]:
                    pos[i] = LANE_PHASES.index(ph)
                    if ph == until:
                        return

        # ungated lanes up to the phases other lanes wait for, the DAMSM lane, then each
        # gated lane forked from the origin stream once its source lane's phase is issued
        # (a fork from the origin, never lane -> lane: see _comm / FlatAdam._allreduce)
        for i in order:
            if i not in gates:
                need = [LANE_PHASES.index(g[1]) for k, g in gates.items() if g[0] == i]
                advance(i, LANE_PHASES[min(need)] if need else None)
        if before_join is not None:
            before_join()
        main = torch.cuda.current_stream()
        for i in order:
            if i in gates:
                j, ph = gates[i]
                advance(j, ph)
                main.wait_stream(streams[j])
                streams[i].wait_stream(main)
                advance(i)
        for i in order:
            advance(i)
        self._join(streams)
        Fn.stamp('d_update joined')
        if g_early is not None:
            g_early[:] = g_terms

    def _d_update_one(self, i, imgs, fake_imgs, sent_emb, unpair_sent_emb, class_labels, iter_rec, real=None):
        """One D of d_update (train.py:439-466), a generator yielding after each
        phase (LANE_PHASES) so d_update can fork other lanes behind it; `real`:
        the real-image heads' values when d_real_early already added their
        gradient."""
        real_img, fake_img, netD, optD = imgs[i], fake_imgs[i], self.netsD[i], self.optimizerDs[i]
        disc_class = self.disc_class and i == 2
        if real is not None:
            # the real-image heads were differentiated by d_real_early: add the fake share
            fk = self.d_loss_fake(fake_img, sent_emb, class_labels, netD, disc_class)
            e_real, e_unpair, e_fake = real[0], real[1], fk[0]
            d_loss = fk[0] / 2.0
            if disc_class:
                c_real, c_unpair, c_fake = real[2], real[3], fk[1]
                d_loss = d_loss + fk[1] / 3.0 * self.d_class_coe
        elif disc_class:
            e_real, e_fake, e_unpair, c_real, c_fake, c_unpair = self.d_loss_class(
                real_img, fake_img, sent_emb, unpair_sent_emb, class_labels, netD)
            d_loss = e_real + (e_fake + e_unpair) / 2.0 + (c_real + c_fake + c_unpair) / 3.0 * self.d_class_coe
        else:
            e_real, e_fake, e_unpair = self.d_loss(real_img, fake_img, sent_emb, unpair_sent_emb, netD)
            d_loss = e_real + (e_fake + e_unpair) / 2.0
        Fn.stamp('D%d loss forward' % i)
        if real is None:
            optD.zero_grad()
        d_loss.backward(inputs=optD.params)
        Fn.stamp('D%d loss backward' % i)
        yield 'loss'
        optD.step()
        Fn.stamp('D%d adam' % i)
        yield 'adam'
        d_loss_gp = self.MA_gradient_penalty(real_img, sent_emb, netD, disc_class)
        Fn.stamp('D%d gp forward + grad' % i)
        optD.zero_grad()
        d_loss_gp.backward(inputs=optD.params)
        Fn.stamp('D%d gp backward' % i)
        yield 'gp'
        optD.step()
        Fn.stamp('D%d gp adam' % i)
        yield 'gpadam'
        if iter_rec:
            self.records['errD_%d/real_sent' % i] = e_real.detach()
            self.records['errD_%d/fake_sent' % i] = e_fake.detach()
            self.records['errD_%d/unpair_sent' % i] = e_unpair.detach()
            self.records['errD_%d/d_loss_gp' % i] = d_loss_gp.detach()
            if disc_class:
                self.records['errD_%d/real_class' % i] = c_real.detach()
                self.records['errD_%d/fake_class' % i] = c_fake.detach()
                self.records['errD_%d/mismatch_class' % i] = c_unpair.detach()

    def damsm_early(self, fake_imgs, sent_emb, words_emb, attr_emb, class_ids, batch_size, match_labels, cap_lens):
        """The DAMSM branch of g_update (image encoder forward + the three
        matching losses), issued on its own stream lane right after the
        generator's forward so it runs concurrently with d_update.  It reads
        only the fake images, the text embeddings and the frozen encoder --
        nothing d_update changes -- so its values are exactly the ones g_update
        would compute after d_update (train.py:490); the lane is joined in
        g_update and the losses enter g_loss there.

        Its backward is issued here too (DAMSM_GRAD_EARLY): g_loss is linear in
        the DAMSM terms (train.py:493, g_loss += DAMSM_coe * (s + w + a)), so
        their gradient w.r.t. the 256-px fake image -- the losses' backward and
        the Inception-v3 input-gradient pass -- depends on nothing d_update
        computes.  It runs on this lane beside the discriminator updates and
        g_update's backward only adds it at the image (the same sum, one
        accumulation order apart), instead of running it behind the D passes
        on the step's critical path.  Returns (w, s, a, dfake or None)."""
        streams = self._side_streams(len(self.netsD) + 1)
        with self._on(streams[-1]):
            Fn.stamp('DAMSM start')
            img = fake_imgs[-1]
            grad_early = DAMSM_GRAD_EARLY and img.requires_grad
            attr = attr_emb
            if grad_early:
                # aliases whose autograd nodes live on this lane: autograd.grad stops at
                # them, so the gradients they capture make no stream of the generator's
                # (main) wait for this lane -- only g_update's backward, through the
                # aliases, joins them
                img = img.view_as(img)
                if attr_emb is not None and attr_emb.requires_grad:
                    # a_loss = sent_loss(cnn_code, attrs_emb) (train.py:432) with attrs_emb
                    # the trainable ATTR_Enhance's output (train.py:193-194): g_loss.backward()
                    # trains ATTR_Enhance through it too, so its gradient is captured here
                    attr = attr_emb.view_as(attr_emb)
            w, s, a = self.DAMSM_loss(img, sent_emb, words_emb, attr, class_ids, batch_size,
                                      match_labels, cap_lens, self.image_encoder)
            Fn.stamp('DAMSM forward')
            dfake = None
            if grad_early:
                leaves = (img, attr) if attr is not attr_emb else (img,)
                grads = torch.autograd.grad(self.DAMSM_coe * (s + w + a), leaves, allow_unused=True)
                w, s, a = w.detach(), s.detach(), a.detach()
                Fn.stamp('DAMSM backward')
                dfake = [(al, g) for al, g in zip(leaves, grads) if g is not None]   # (alias, gradient there)
        return w, s, a, dfake

    def _g_term(self, i, fake_imgs, sent_emb, class_labels, iter_rec):
        """The generator's adversarial term through D i (train.py:477-489)."""
        fake_img, netD = fake_imgs[i], self.netsD[i]
        Fn.stamp('gD%d start' % i)
        n_early = GTERM_GRAD_EARLY if GTERM_GRAD_EARLY >= 0 else len(self.netsD)
        grad_early = i < n_early and fake_img.requires_grad and torch.is_grad_enabled()
        if grad_early:
            # an alias whose autograd node lives on this lane (as in damsm_early):
            # autograd.grad stops at it, g_update's backward enters through it
            fake_img = fake_img.view_as(fake_img)
        if self.disc_class and i == 2:
            errG, errG_class = self.g_loss_class(fake_img, sent_emb, class_labels, netD)
            term = errG + errG_class * self.g_class_coe
        else:
            errG = self.g_loss(fake_img, sent_emb, netD)
            term = errG
        Fn.stamp('gD%d forward' % i)
        if iter_rec:
            self.records['errG/G_%d_fake_sent' % i] = errG.detach()
            if self.disc_class and i == 2:
                self.records['errG/G_%d_fake_class' % i] = errG_class.detach()
        if grad_early:
            (dfake,) = torch.autograd.grad(term, fake_img)
            Fn.stamp('gD%d input grad' % i)
            return EarlyTerm(term.detach(), fake_img, dfake)
        return term

    def g_update(self, fake_imgs, sent_emb, words_emb, attr_emb, class_ids, batch_size, match_labels, cap_lens,
                 class_labels, iter_rec=False, damsm=None, terms=None):
        """train.py:471-502 (`damsm`: the losses from damsm_early, `terms`: the
        per-D terms from d_update(g_early=...); else computed here)."""
        nD = len(self.netsD)
        streams = self._side_streams(nD + 1)
        if not terms:
            terms = []
            for i in range(nD):
                with self._on(streams[i]):
                    terms.append(self._g_term(i, fake_imgs, sent_emb, class_labels, iter_rec))
        if damsm is None:
            with self._on(streams[nD]):
                Fn.stamp('DAMSM start')
                damsm = self.DAMSM_loss(fake_imgs[-1], sent_emb, words_emb, attr_emb, class_ids,
                                        batch_size, match_labels, cap_lens, self.image_encoder)
                Fn.stamp('DAMSM forward')
        w_loss, s_loss, a_loss = damsm[:3]
        dfake = damsm[3] if len(damsm) > 3 else None
        self._join(streams)
        Fn.stamp('g_update forwards joined')
        g_loss = _term_value(terms[0])
        for t in terms[1:]:
            g_loss = g_loss + _term_value(t)
        g_adv = g_loss
        g_loss = g_loss + self.DAMSM_coe * (s_loss + w_loss + a_loss)
        if iter_rec:
            self.records['errG/s_loss'] = s_loss.detach()
            self.records['errG/w_loss'] = w_loss.detach()
            self.records['errG/a_loss'] = a_loss.detach()
        if Fn.STAMPS is not None:   # diagnostics: when each fake image's gradient is complete
            for i, f in enumerate(fake_imgs):
                f.register_hook(lambda g, i=i: (Fn.stamp('dfake%d ready' % i), g)[1])
        gen = getattr(self.netG, 'module', self.netG)
        if not getattr(self, '_g_zeroed', False):
            self.zero_grad_G()
        self._g_zeroed = False
        # only the optimised parameters' gradients are formed: train.py's
        # g_loss.backward() also fills the D parameters' .grad, but d_update
        # zeroes those before every use (train.py:451,457), and the GP's
        # interpolated-image gradient is never read -- skipping them changes no
        # parameter and saves the D weight-gradient passes
        self._g_backward(terms, dfake, g_adv, g_loss, s_loss, w_loss, a_loss)
        if getattr(gen, 'side_stream', None) is not None:
            # the branch's backward nodes ran on the lane: their direct p.grad writes
            # (functional._grad_sink) are not among autograd's leaf-stream syncs
            self._join([gen.side_stream])
        Fn.stamp('G backward (D, DAMSM, G)')
        self.optimizerG.step()
        Fn.stamp('G adam')
        return g_loss.detach()

    def zero_grad_G(self):
        """optimizerG.zero_grad() (train.py:498), ordered before the generator
        branch's lane as well: that lane's backward nodes write parameter
        gradients straight into the flat buffer (functional._grad_sink), and
        autograd syncs a node only with the producers of its input gradients --
        a node whose input gradient was made on the lane itself (the 64-px
        image's, GTERM_GRAD_EARLY) would otherwise accumulate before the zero
        fill on the main stream lands."""
        self.optimizerG.zero_grad()
        gen = getattr(self.netG, 'module', self.netG)
        if getattr(gen, 'side_stream', None) is not None:
            gen.side_stream.wait_stream(torch.cuda.current_stream())

    def _g_backward(self, terms, dfake, g_adv, g_loss, s_loss, w_loss, a_loss):
        if any(isinstance(t, EarlyTerm) for t in terms):
            # per-D terms differentiated on their lanes enter at their image aliases
            roots, grads = _backward_roots(terms)
            if dfake is not None:
                for alias, g in dfake:
                    roots.append(alias)
                    grads.append(g)
            else:
                roots.append(self.DAMSM_coe * (s_loss + w_loss + a_loss))
                grads.append(None)
            torch.autograd.backward(roots, grads, inputs=self.optimizerG.params)
        elif dfake is not None:
            # the DAMSM terms' share, computed by damsm_early, enters at its aliases of the
            # 256-px image and of ATTR_Enhance's attribute embedding
            torch.autograd.backward([g_adv] + [al for al, _ in dfake], [None] + [g for _, g in dfake],
                                    inputs=self.optimizerG.params)
        else:
            g_loss.backward(inputs=self.optimizerG.params)

    # ---------------------------------------------------- failure checks --
    CHECK_EVERY = D.CHECK_EVERY   # steps between checks of the collectives' error state (each check synchronises)

    @staticmethod
    def check_collectives():
        """Raise if a SyncBN peer-write reduction timed out (EEGAN_SYNCBN_PEER):
        called every CHECK_EVERY steps / replays and before state is saved."""
        D.check_collectives()

    def state_dict(self):
        """Optimizer state for checkpoints (collectives checked first: a
        desynchronised rank must not write a checkpoint)."""
        self.check_collectives()
        return {'optimizerG': self.optimizerG.state_dict(),
                'optimizerDs': [o.state_dict() for o in self.optimizerDs]}

    # -------------------------------------------------------- inner step --
    def encode_text(self, batch):
        """train.py:169-184: 5 frozen text-encoder calls (captions, 3 attributes, unpaired)."""
        enc = self.text_encoder
        caps, ucaps = batch['caps'], batch['unpair_caps']
        if batch.get('max_len') is not None and caps.shape == ucaps.shape:
            # the frozen encoder is per-caption: captions + unpaired captions as
            # one batch, the three attribute phrases as another (2 calls, not 5)
            B = caps.shape[0]
            with torch.no_grad():
                w2, s2 = enc(torch.cat([caps, ucaps], 0), torch.cat([batch['cap_lens'].reshape(-1),
                                                                     batch['unpair_cap_lens'].reshape(-1)], 0),
                             None, max_len=batch['max_len'])
                at = batch['attrs'][:, :self.max_attr_nums, :]
                _, sa = enc(at.reshape(B * at.shape[1], at.shape[2]), batch['attrs_len'][:, :self.max_attr_nums].reshape(-1),
                            None, max_len=at.shape[2])
            return w2[:B], s2[:B], sa.reshape(B, at.shape[1], -1), s2[B:]
        with torch.no_grad():
            words, sent = enc(batch['caps'], batch['cap_lens'], None, max_len=batch.get('max_len'))
            attrs = []
            for i in range(self.max_attr_nums):
                _, a = enc(batch['attrs'][:, i, :], batch['attrs_len'][:, i], None, max_len=batch['attrs'].shape[2])
                attrs.append(a)
            attrs = torch.stack(attrs, dim=1)
            _, unpair = enc(batch['unpair_caps'], batch['unpair_cap_lens'], None,
                            max_len=batch['unpair_caps'].shape[1])
        return words, sent, attrs, unpair

    def train_step(self, batch, noise=None, emb=None, iter_rec=False):
        """One iteration of train.py:163-206 on a device-resident batch."""
        B = self.batch_size
        dev = self.device
        Fn.stamp('start')
        comm = self._comm_lanes()
        main = torch.cuda.current_stream()
        for cs in comm:   # forked from the origin stream at the start (graph capture: never from a lane)
            cs.wait_stream(main)
        for o in (self.optimizerDs[-1], self.optimizerG) if comm else ():
            o.comm_origin = main
        words, sent, attrs, unpair = emb if emb is not None else self.encode_text(batch)
        Fn.stamp('text encode')
        class_labels = None
        if self.disc_class:
            class_labels = prepare_class_labels(B, self.class_nums, batch['cls_ids'], dev)
        if noise is None:
            noise = torch.randn(B, 100, device=dev)
        real = {}
        if DREAL_EARLY and self.use_streams:
            lanes = self._side_streams(len(self.netsD) + 1, fork=False)   # (the full set: never re-created mid-step)
            for i in DREAL_EARLY:
                if 0 <= i < len(self.netsD):
                    # on the D's own lane, or on the DAMSM lane (idle until the generator's
                    # images exist) with d_update's fork ordered behind it
                    lane = lanes[i] if DREAL_LANE == 'own' else lanes[-1]
                    lane.wait_stream(main)
                    with self._on(lane):
                        real[i] = self.d_real_early(i, batch['imgs'], sent, unpair, class_labels)
        _, attn_attr_emb = self.attr_enhance(sent, attrs)
        attn_attr_emb = self.attr_enhance.module.attr_merge(attn_attr_emb)
        gen = getattr(self.netG, 'module', self.netG)
        if hasattr(gen, 'side_stream'):
            # stage 2-3 Cum_Block / image branches on D64's lane, idle until d_update forks
            gen.side_stream = self._side_streams(len(self.netsD) + 1, fork=False)[0] if GEN_SIDE else None
        fake_imgs = self.netG(noise, sent, attn_attr_emb)
        if getattr(gen, 'side_stream', None) is not None:
            # the generator's gradients are zeroed now (nothing before g_update
            # writes them), so g_update's backward nodes on the branch's lane can
            # start as soon as their input gradients are ready -- beside the
            # largest discriminator's update -- instead of after it
            self.zero_grad_G()
            self._g_zeroed = True
        Fn.stamp('ATTR + G forward')
        if real and DREAL_LANE != 'own':
            main.wait_stream(self._side_streams(len(self.netsD) + 1, fork=False)[-1])
        _, _, match_labels = prepare_labels(B, dev)
        cls_ids = batch.get('cls_ids')  # train.py:490 passes class ids to DAMSM_loss even without USE_CLASS
        damsm = []
        early = DAMSM_EARLY and self.use_streams

        def issue_damsm():
            damsm[:] = self.damsm_early(fake_imgs, sent, words, attn_attr_emb, cls_ids, B, match_labels,
                                        batch['cap_lens'])
        if early and LANE_ORDER != 'rev':
            issue_damsm()
        terms = [] if (G_EARLY and self.use_streams) else None
        self.d_update(batch['imgs'], fake_imgs, sent, unpair, class_labels, iter_rec, g_early=terms,
                      before_join=issue_damsm if early and LANE_ORDER == 'rev' else None, real=real)
        damsm = damsm or None
        g = self.g_update(fake_imgs, sent, words, attn_attr_emb, cls_ids, B, match_labels, batch['cap_lens'],
                          class_labels, iter_rec, damsm=damsm, terms=terms)
        self._join(comm)   # (each optimizer step already waited for its lane)
        Fn.stamp('end')
        self._steps = getattr(self, '_steps', 0) + 1
        if self._steps % self.CHECK_EVERY == 0 and not torch.cuda.is_current_stream_capturing():
            self.check_collectives()
        return fake_imgs, g


class StepGraph(object):
    """The whole train_step captured once as a HIP graph (torch.cuda.CUDAGraph
    is hipGraph on ROCm) and replayed: each iteration is one graph launch
    instead of ~3000 kernel launches issued through Python autograd, which
    otherwise bounds the step on the host.

    Requirements the step already meets: no host reads of device values, a
    batch held in fixed device storage (refill it in place between replays),
    noise drawn inside the graph (graph-safe philox offsets), Adam bias
    corrections from device step counters, and weight packs refreshed by
    kernels that are part of the graph.  Learning rates are baked in.
    """

    def __init__(self, trainer, batch, warmup=2, timer=None, keep_graph=False, **step_kw):
        from . import functional as Fn
        side = new_stream(torch.cuda.current_device())
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(warmup):
                trainer.train_step(batch, **step_kw)
        torch.cuda.current_stream().wait_stream(side)
        # keep_graph: the hipGraph stays inspectable after instantiation (node counts, tools/probe)
        self.graph = torch.cuda.CUDAGraph(keep_graph=keep_graph)
        prev, Fn.TIMER = Fn.TIMER, timer
        # with a process group the RCCL collectives (SyncBN statistics, DAMSM
        # gathers, gradient buckets) are captured too; thread-local capture
        # keeps the process group's watchdog thread from invalidating it
        mode = 'thread_local' if D.collective() else 'global'
        dbg = os.environ.get('EEGAN_DEBUG_CAPTURE') == '1'

        def capture():
            # captured on the stream the warm-up ran on: per-stream side streams
            # (weight gradients) were created there, outside the capture
            if dbg:
                print('StepGraph: capture begin', file=sys.stderr, flush=True)
            with torch.cuda.graph(self.graph, stream=side, capture_error_mode=mode):
                self.out = trainer.train_step(batch, **step_kw)
                if dbg:
                    print('StepGraph: step recorded, ending capture', file=sys.stderr, flush=True)
            if dbg:
                print('StepGraph: capture ended (instantiated)', file=sys.stderr, flush=True)

        try:
            stack_mb = int(os.environ.get('EEGAN_CAPTURE_STACK_MB', '0'))
            if stack_mb > 0:
                # capture + instantiate on a thread with a large stack (the runtime's
                # graph walk recurses per dependency edge)
                import threading
                err = []

                def run():
                    try:
                        torch.cuda.set_device(side.device)
                        capture()
                    except BaseException as e:  # re-raised on the caller's thread
                        err.append(e)
                old = threading.stack_size(stack_mb << 20)
                try:
                    th = threading.Thread(target=run)
                    th.start()
                    th.join()
                finally:
                    threading.stack_size(old)
                if err:
                    raise err[0]
            else:
                capture()
        finally:
            Fn.TIMER = prev

    # Replays kept in flight.  Back-to-back graph launches fill the HW queues
    # (the host then blocks inside hipGraphLaunch, `host_issue_ms_per_step` ~
    # the GPU time) and the next replay's packets queue up beside the running
    # one's: the step's stream lanes then run slower.  Measured on the C2 step
    # (tools/probe/graph_submit.py, profiles/r03_graph_submit.json): 27.4-27.8
    # ms per step unpaced or with 2-3 replays in flight, 25.8-26.0 ms when each
    # replay is submitted after the previous one finished (one replay from an
    # idle GPU: 25.6 ms); submitting one replay costs 6.3 ms of host time
    # (GPU blocked, 2,390 nodes / 2,417 edges), so it overlaps the replay it
    # launches.  With depth d the host waits for replay k-d before launching
    # replay k.  EEGAN_REPLAY_DEPTH=0: unpaced.
    DEPTH = int(os.environ.get('EEGAN_REPLAY_DEPTH', '1'))

    def replay(self):
        self._n = getattr(self, '_n', 0) + 1
        if self._n % Trainer.CHECK_EVERY == 0:
            Trainer.check_collectives()
        if self.DEPTH > 0:
            q = getattr(self, '_inflight', None)
            if q is None:
                q = self._inflight = []
            while len(q) >= self.DEPTH:
                q.pop(0).synchronize()
        self.graph.replay()
        if self.DEPTH > 0:
            ev = torch.cuda.Event()
            ev.record()
            self._inflight.append(ev)
        return self.out
