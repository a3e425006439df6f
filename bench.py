#!/usr/bin/env python
"""Benchmark: EE-GAN data-parallel G+D training step on MI355X.

Metric (BASELINE.json): train images/sec at 256x256 CUB, full 3-stage G+D
step (text encode x5 -> ATTR_Enhance -> G -> d_update x3 (hinge + class +
MA gradient penalty, 2 Adam steps per D) -> g_update (3 D's + Inception-v3
DAMSM words/sent losses, 1 Adam step)).  Workload C2: CUB GF=DF=32, batch 16
per GPU, bf16 activations / fp32 master weights, synthetic data, random
initialised weights (no datasets/checkpoints offline).

    python bench.py [--gpus N] [--steps K] [--warmup W]
        (N > 1: starts `torch.distributed.run --standalone --nproc-per-node N
        bench.py ...` as a child job, one rank per GPU, and relays rank 0's line)
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU, RCCL)

Prints ONE JSON line on rank 0 (see the repo README / task contract), with a
`roofline` object for the dominant conv kernel family (by summed dispatch
time: forward, backward-data or weight-gradient implicit GEMM, bf16 MFMA),
timed per dispatch with HIP events, its PMC traffic and MFMA-busy figures
from the committed rocprofv3 summary of the same config, and a
`cpu_baseline` object: the CPU oracle (oracle/, a PyTorch-CPU restatement of
the reference step) timed on the host on a bounded sample.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, 'ee-gan_amd'))
sys.path.insert(0, REPO)

# bench.py sets each rank's device and starts the process group itself
# (eegan_hip.dist.init_from_env): no import-time pinning (eegan_hip.launch)
os.environ.setdefault('EEGAN_AUTO_DIST', '0')

import torch  # noqa: E402

CONFIGS = {
    # name: (dataset, GF=DF, per-GPU batch, class_num (0 = no class head))
    'C2': ('CUB-200', 32, 16, 200),
    'C3': ('Oxford-102', 48, 32, 102),
    'C4': ('MS-COCO', 64, 8, 0),
    'C5': ('CUB-200', 32, 32, 200),
    'T8': ('CUB-200 (test size)', 8, 4, 10),   # parity tests only, not a bench line
}
# whole-step ceilings per GPU (BASELINE.md roofline table: algorithmic FLOPs /
# bf16 conv-path bytes per image over 2.5 PFLOP/s and 8 TB/s): (MFMA, HBM) img/s
CEILINGS = {'C2': (8300.0, 6300.0), 'C3': (3760.0, 4300.0), 'C4': (2140.0, 2520.0), 'C5': (8300.0, 6500.0)}
MFMA_PEAK_TFLOPS = 2500.0   # dense bf16 (MI355X_MICROARCH.md)
HBM_PEAK_GBS = 8000.0


def build(cfg_name, device, sim_coe=0.05):
    import models
    import DAMSM
    from sync_batchnorm import DataParallelWithCallback
    from eegan_hip.trainer import Trainer
    _, W, B, ncls = CONFIGS[cfg_name]
    torch.manual_seed(3407)
    G = DataParallelWithCallback(models.Gen(W, 100).to(device))
    A = DataParallelWithCallback(models.ATTR_Enhance().to(device))
    disc_class = ncls > 0
    Ds = [DataParallelWithCallback(models.Dis64(W).to(device)), DataParallelWithCallback(models.Dis128(W).to(device)),
          DataParallelWithCallback(models.Dis256(W, disc_class, max(ncls, 1)).to(device))]
    # zero-initialised gammas/heads of the reference would make most branches
    # dead at step 0; use small non-zero values so every kernel does its work
    with torch.no_grad():
        for m in [G, A] + Ds:
            for n, p in m.named_parameters():
                if n.endswith('gamma'):
                    p.fill_(0.5)
                elif 'linear2' in n:
                    p.normal_(0, 0.02)
    enc_img = DAMSM.CNN_ENCODER(256).to(device).eval()
    enc_txt = DAMSM.RNN_ENCODER(5450, nhidden=256).to(device).eval()
    for p in enc_txt.parameters():
        p.requires_grad = False
    T = Trainer(G, A, Ds, enc_img, enc_txt, B, disc_class=disc_class, class_nums=max(ncls, 1), class_coe=10.0,
                sim_coe=sim_coe, device=device)
    return T, B, ncls


def _lib_sha():
    import hashlib
    h = hashlib.sha256()
    with open(os.path.join(REPO, 'ee-gan_amd', 'eegan_hip', 'libeegan_hip.so'), 'rb') as f:
        h.update(f.read())
    return h.hexdigest()[:16]


def pmc_summary(config):
    """The newest committed rocprofv3 summary of workload `config`
    (profiles/rNN_<config>_families.json, tools/gpu_profile.sh +
    tools/rocprof_families.py: kernel-trace pass plus one PMC pass per
    counter).  Returns (summary dict, path, current) where current says the
    summary was taken with the libeegan_hip.so this run loaded (its sha256);
    (None, None, False) when no summary of this config exists."""
    import glob
    files = sorted(glob.glob(os.path.join(REPO, 'profiles', 'r*_%s_families.json' % config)))
    if not files:
        return None, None, False
    with open(files[-1]) as f:
        summ = json.load(f)
    try:
        current = summ.get('lib_sha256_16') == _lib_sha()
    except OSError:
        current = False
    return summ, 'profiles/' + os.path.basename(files[-1]), current


def conv_path_hbm_frac(fams):
    """Whole conv path (fwd + bwd-data + wgrad families): PMC HBM bytes over
    kernel time over the 8 TB/s peak (north_star's definition).
    Counts every byte the counters saw, wasted re-reads included."""
    tot_b = tot_s = 0.0
    for k in ('conv_fwd', 'conv_bwd_data', 'conv_bwd_weight'):
        f = fams.get(k, {})
        if not f.get('hbm_bytes_per_call') or not f.get('calls'):
            return None
        tot_b += f['hbm_bytes_per_call'] * f['calls']
        tot_s += f['total_ms'] * 1e-3
    return round(tot_b / tot_s / 1e9 / HBM_PEAK_GBS, 4) if tot_s else None


def host_submit_ms(step, reps=3):
    """Host time of submitting one step (graph replay) while the GPU is held
    by a ~0.3 s spin kernel: the pure submission cost, without the queue
    back-pressure that makes the host wait during back-to-back replays."""
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        torch.cuda._sleep(int(2.4e9 * 0.3))
        t0 = time.perf_counter()
        step()
        ts.append((time.perf_counter() - t0) * 1e3)
    torch.cuda.synchronize()
    return round(sorted(ts)[len(ts) // 2], 3)


def _cpu_model():
    try:
        with open('/proc/cpuinfo') as f:
            for line in f:
                if line.startswith('model name'):
                    return line.split(':', 1)[1].strip()
    except OSError:
        pass
    return 'unknown'


def cpu_baseline(seconds_budget=30.0):
    """The CPU oracle (oracle.eegan_oracle, the PyTorch-CPU restatement of the
    reference step, pinned to golden vectors captured from the reference)
    timed on the host: BASELINE.md's CPU plan -- W=32, B=4, the five frozen
    text-encoder calls (train.py:169-184) inside the step, the full 3-stage
    step (incl. the Inception-v3 restatement) and the C1 stage-1 slice;
    warm-ups until three consecutive steps agree within 5 % (at most 15), then the median of
    at least 10 steps; threads = the affinity set capped by the box's CPU
    share (stated as `threads_reason`)."""
    from oracle import eegan_oracle as O
    from oracle.seeding import seeded_state, synthetic_batch
    import models
    import DAMSM
    # the host cores this process may use: the affinity set, capped by the
    # scheduler's share when the environment states one (OMP_NUM_THREADS: the
    # GPU box's affinity mask spans the whole machine, its CPU share is 16).
    # Measured by the parent (cpu_baseline_child): here OpenMP's bound initial
    # thread already narrowed this process's own mask to one core
    affinity = int(os.environ.get('EEGAN_CPU_AFFINITY') or len(os.sched_getaffinity(0)))
    share = int(os.environ.get('EEGAN_CPU_SHARE') or 0)
    torch.set_num_threads(min(affinity, share) if share > 0 else affinity)
    B, W, ncls = 4, 32, 200
    spec = lambda m: [(k, tuple(v.shape)) for k, v in m.state_dict().items()]  # noqa: E731
    sd_e = seeded_state(spec(DAMSM.CNN_ENCODER(256)), 9)
    sd_t = seeded_state(spec(DAMSM.RNN_ENCODER(5450, nhidden=256)), 10)
    batch = synthetic_batch(B, seed=5, class_num=ncls)
    enc = lambda x: O.cnn_encoder(sd_e, x)  # noqa: E731

    def encode_text():
        with torch.no_grad():
            words, sent = O.rnn_encoder(sd_t, batch['caps'], batch['cap_lens'])
            attrs = torch.stack([O.rnn_encoder(sd_t, batch['attrs'][:, i], batch['attrs_len'][:, i])[1]
                                 for i in range(3)], 1)
            _, unpair = O.rnn_encoder(sd_t, batch['unpair_caps'], batch['unpair_cap_lens'])
        return words, sent, attrs, unpair

    def timed(stages, budget):
        sd_g = seeded_state(spec(models.Gen(W, 100)), 1)
        sd_a = seeded_state(spec(models.ATTR_Enhance()), 2)
        nd = 3 if stages == 3 else 1
        sd_ds = [seeded_state(spec(m), 3 + i) for i, m in enumerate([models.Dis64(W), models.Dis128(W),
                                                                      models.Dis256(W, True, ncls)][:nd])]
        nets = O.OracleNets(sd_g, sd_a, sd_ds, W, W, True, ncls)
        og, ods = O.make_adams(nets)
        # warm-ups until three consecutive steps agree within 5 % (the first steps run up to
        # 2x slower: allocator, thread-pool and page warm-up), at most 15
        hist, warm = [], 0
        while warm < 15:
            t0 = time.time()
            O.train_step(nets, og, ods, batch, encode_text(), enc, stages=stages)
            hist.append(time.time() - t0)
            warm += 1
            print('bench: cpu baseline (%d stage%s) warm-up %d: %.2f s' % (stages, 's' if stages > 1 else '', warm,
                                                                         hist[-1]), file=sys.stderr, flush=True)
            if len(hist) >= 3 and max(hist[-3:]) <= 1.05 * min(hist[-3:]):
                break
        times = []
        t_end = time.time() + budget
        while len(times) < 10 or (time.time() < t_end and len(times) < 20):
            t0 = time.time()
            O.train_step(nets, og, ods, batch, encode_text(), enc, stages=stages)
            times.append(time.time() - t0)
            print('bench: cpu baseline (%d stage%s) step %d: %.2f s' % (stages, 's' if stages > 1 else '',
                                                                       len(times), times[-1]), file=sys.stderr,
                  flush=True)
        spread = (max(times) - min(times)) / min(times)
        times.sort()
        # interquartile spread: one step slowed by another job on the shared host moves
        # max/min, not the quartiles (nor the median that is reported)
        q1, q3 = times[len(times) // 4], times[(3 * len(times)) // 4]
        warmups[stages] = (warm, spread, (q3 - q1) / q1)
        return B / times[len(times) // 2], len(times)

    warmups = {}
    try:   # before the first parallel op (the child process runs nothing else first)
        torch.set_num_interop_threads(1)
    except RuntimeError:
        pass
    full, n_full = timed(3, seconds_budget)
    c1, n_c1 = timed(1, 0.25 * seconds_budget)
    return {'value': full, 'unit': 'images/sec', 'cores': torch.get_num_threads(), 'kind': 'port',
            'affinity_cores': affinity, 'cpu_model': _cpu_model(),
            'threads_reason': ('OMP_NUM_THREADS=%d: the CPU share the GPU box grants this process; its affinity mask '
                               'spans all %d cores of the host, shared with the other GPUs\' jobs' % (share, affinity))
            if 0 < share < affinity else 'all affinity cores',
            'sample': 'oracle train_step (full 3-stage, W=32, B=4: 5 text-encoder calls, G, 3 x d_update incl. '
                      'the gradient penalty, g_update incl. the Inception-v3 restatement), median of %d steps after '
                      '%d warm-ups (until three consecutive steps agreed within 5%%); max/min spread of the timed '
                      'steps %.2f' % (n_full, warmups[3][0], warmups[3][1]),
            'binding': 'own process; OMP_PROC_BIND=%s OMP_PLACES=%s, %d intra-op threads, %d inter-op' % (
                os.environ.get('OMP_PROC_BIND', 'unset'), os.environ.get('OMP_PLACES', 'unset'),
                torch.get_num_threads(), torch.get_num_interop_threads()),
            'timed_spread': round(warmups[3][1], 4),
            'timed_iqr_spread': round(warmups[3][2], 4),
            'c1_stage1': {'value': c1, 'unit': 'images/sec', 'sample': 'C1 stage-1 slice (img_64, Dis64, DAMSM on '
                                                                       'img_64), B=4, median of %d steps after %d '
                                                                       'warm-ups' % (n_c1, warmups[1][0])}}


def launcher_argv(n, argv):
    """The child job `python bench.py --gpus N` starts when no launcher set
    WORLD_SIZE: torch.distributed.run with one rank per GPU of this node and
    a rendezvous store that binds its own port (--standalone: c10d on port 0)
    on 127.0.0.1 -- the same per-rank bench.py, unchanged arguments."""
    return [sys.executable, '-m', 'torch.distributed.run', '--standalone', '--local-addr', '127.0.0.1',
            '--nnodes=1', '--nproc-per-node', str(n), os.path.abspath(__file__)] + list(argv)


def launch_ranks(n, argv):
    """Run the N-rank job as a child process (never exec: nothing here has
    touched the GPU, and the child is a fresh interpreter), relay rank 0's
    JSON line to stdout (anything else the ranks print to stdout goes to
    stderr) and return the job's exit status."""
    import subprocess
    cmd = launcher_argv(n, argv)
    print('bench: --gpus %d without WORLD_SIZE: launching %s' % (n, ' '.join(cmd)), file=sys.stderr, flush=True)
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True)
    line = None
    for raw in p.stdout:
        try:
            rec = json.loads(raw)
        except ValueError:
            rec = None
        if isinstance(rec, dict) and 'metric' in rec:
            line = raw.strip()
        else:
            sys.stderr.write(raw)
            sys.stderr.flush()
    rc = p.wait()
    if line is not None:
        print(line, flush=True)
    if rc == 0 and line is None:
        print('bench: the %d-rank job printed no result line' % n, file=sys.stderr, flush=True)
        return 1
    return rc


def cpu_baseline_child(seconds):
    """cpu_baseline() in a fresh process of its own (no HIP runtime threads,
    OpenMP threads bound to cores from the start: OMP_PROC_BIND / OMP_PLACES
    only act before OpenMP starts, which in this process happened long ago),
    started after the GPU measurement; returns its JSON object."""
    import subprocess
    affinity = len(os.sched_getaffinity(0))
    share = int(os.environ.get('OMP_NUM_THREADS') or 0)
    threads = min(affinity, share) if share > 0 else affinity
    env = dict(os.environ, OMP_PROC_BIND='close', OMP_PLACES='cores', OMP_NUM_THREADS=str(threads),
               EEGAN_CPU_AFFINITY=str(affinity), EEGAN_CPU_SHARE=str(share))
    r = subprocess.run([sys.executable, os.path.abspath(__file__), '--cpu-baseline-only',
                        '--cpu-seconds', str(seconds)], env=env, stdout=subprocess.PIPE, text=True, timeout=900)
    lines = [l for l in r.stdout.splitlines() if l.startswith('{')]
    if r.returncode != 0 or not lines:
        return {'error': 'cpu baseline child exited %d' % r.returncode}
    return json.loads(lines[-1])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=10)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--config', default='C2', choices=sorted(CONFIGS))
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--cpu-seconds', type=float, default=30.0)
    ap.add_argument('--cpu-baseline-only', action='store_true', help=argparse.SUPPRESS)
    ap.add_argument('--no-timer', action='store_true', help='diagnostic: skip the roofline timing pass')
    ap.add_argument('--timing-steps', type=int, default=2, help='eager steps of the roofline timing pass')
    ap.add_argument('--op-log', help='diagnostic: write the timing pass\'s conv / GEMM ops (issue order, shape, '
                                     'algorithmic FLOPs / bytes) as JSON, for tools/rocprof_families.py --ops')
    ap.add_argument('--graph', default='auto', choices=['auto', 'on', 'off'],
                    help='replay the step as one captured HIP graph (auto: on; N > 1 needs the own RCCL communicators)')
    args = ap.parse_args()
    if args.cpu_baseline_only:   # the child of cpu_baseline_child(): no GPU
        print(json.dumps(cpu_baseline(args.cpu_seconds)), flush=True)
        return
    if args.gpus > 1 and 'WORLD_SIZE' not in os.environ:
        # `python bench.py --gpus N` without a launcher: start the N ranks as a child job
        # (one process per GPU, RCCL) before this process touches the GPU; no exec
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    if int(os.environ.get('WORLD_SIZE', '1')) != args.gpus:
        raise SystemExit('bench: --gpus %d but WORLD_SIZE=%s: refusing to report a number for another GPU '
                         'count' % (args.gpus, os.environ.get('WORLD_SIZE', '1')))

    from eegan_hip import dist as D
    from eegan_hip import functional as Fn
    from eegan_hip.synthetic import make_batch
    local_rank = int(os.environ.get('LOCAL_RANK', '0'))
    if os.environ.get('EEGAN_SHARE_GPU') == '1':   # rehearsal only: several ranks on one GPU (gloo)
        local_rank %= torch.cuda.device_count()
    torch.cuda.set_device(local_rank)
    device = torch.device('cuda', local_rank)
    rank, world = D.init_from_env()
    if world != args.gpus:
        raise SystemExit('bench: --gpus %d but the job has %d rank(s) (WORLD_SIZE=%s): refusing to report a '
                         'number for another GPU count' % (args.gpus, world, os.environ.get('WORLD_SIZE')))
    T, B, ncls = build(args.config, device)
    batch = make_batch(B, device, seed=3407 + rank, class_num=ncls, with_class=True, id_offset=rank * B)

    # the whole step, collectives included (own per-lane RCCL communicators,
    # eegan_hip.rccl), is one captured HIP graph on every rank
    # (EEGAN_GRAPH_DIST=0: eager steps when N > 1)
    use_graph = args.graph == 'on' or (args.graph == 'auto' and (
        world == 1 or (bool(D.COMMS) and os.environ.get('EEGAN_GRAPH_DIST', '1') == '1')))
    graph_error = None
    from eegan_hip.trainer import StepGraph
    if use_graph:
        # the eager timing pass after the capture re-enters AccumulateGrad nodes first seen on the
        # capture stream; torch warns about the stream change, which is harmless here
        torch.autograd.graph.set_warn_on_accumulate_grad_stream_mismatch(False)
        try:
            sg = StepGraph(T, batch, warmup=max(1, args.warmup - 1))   # eager warm-ups, then capture
            step = sg.replay
            step()  # last warm-up = first replay
        except Exception as e:  # capture refused (e.g. a runtime without collective capture): run eagerly
            graph_error = repr(e)[:300]
            print('bench: step graph capture failed, running eagerly: %s' % graph_error, file=sys.stderr,
                  flush=True)
            use_graph = False
            torch.cuda.synchronize()
    if not use_graph:
        def step():
            T.train_step(batch)

        for _ in range(args.warmup):
            step()
    # window markers for tools/rocprof_families.py (a one-thread stamp kernel at both
    # ends of the timed region and of the timing pass), outside the timed region
    from eegan_hip._lib import ops as _ops
    marks = torch.zeros(4, dtype=torch.int64, device=device)

    def mark(i):
        _ops.stamp(marks.data_ptr() + 8 * i, torch.cuda.current_stream().cuda_stream)

    mark(0)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    t_issue = time.perf_counter() - t0   # host time to enqueue the K steps
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    mark(1)
    if world > 1:
        t = torch.tensor([dt], device=device)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        dt = t.item()

    # host cost of submitting one step with the GPU held busy (no queue back-pressure)
    submit_ms = host_submit_ms(step) if use_graph else None

    # roofline timing pass: the same step run eagerly right after the timed
    # region, every conv / GEMM dispatch stamped by its own HIP start/stop
    # events (hipExtLaunchKernel), so host launch gaps are excluded
    timer = None
    per = max(1, args.timing_steps)
    if not args.no_timer:
        timer = Fn.LaunchTimer()
        Fn.TIMER = timer
        # single stream while timing: a dispatch sharing the GPU with another
        # stream's kernels would read longer than its own work
        streams, T.use_streams = T.use_streams, False
        mark(2)
        for _ in range(per):
            T.train_step(batch)
        mark(3)
        T.use_streams = streams
        Fn.TIMER = None
        if args.op_log and rank == 0:   # the timing pass's ops in issue order (per-op PMC table)
            with open(args.op_log, 'w') as f:
                json.dump({'config': args.config, 'timing_steps': per, 'ops': timer.ops}, f)
    kern = timer.summary() if timer is not None else {'conv_fwd': [1, 0.0, 0.0, 1.0]}
    ms = dt / args.steps * 1e3
    value = B * world * args.steps / dt
    # dominant kernel family by time
    dom = max(((k, v) for k, v in kern.items() if k.startswith('conv')), key=lambda kv: kv[1][3])
    kind, (n, fl, nb, tsec) = dom
    achieved = fl / tsec / 1e12
    summ, traffic_src, current = pmc_summary(args.config)
    pfams = (summ or {}).get('families', {})
    pf = pfams.get(kind, {})
    traffic = pf.get('hbm_bytes_per_call')
    fam_out = {}
    for k, v in kern.items():
        e = {'ms_per_step': round(v[3] / per * 1e3, 3), 'TFLOPs': round(v[1] / max(v[3], 1e-12) / 1e12, 1)}
        if k.startswith('conv'):
            n_k = max(v[0], 1)
            e['launches_per_step'] = v[0] // per
            e['algorithmic_bytes_per_launch'] = round(v[2] / n_k)
            e['algorithmic_flops_per_launch'] = round(v[1] / n_k)
            e['frac_of_mfma_peak'] = round(v[1] / max(v[3], 1e-12) / 1e12 / MFMA_PEAK_TFLOPS, 4)
            q = pfams.get(k, {})
            if q.get('hbm_bytes_per_call') and v[2] > 0:
                e['pmc_bytes_per_launch'] = q['hbm_bytes_per_call']
                e['pmc_over_algorithmic'] = round(q['hbm_bytes_per_call'] / max(v[2] / n_k, 1), 3)
            if q.get('mfma_util') is not None:
                e['mfma_busy'] = q['mfma_util']
            if q.get('mfma_busy_cycles_per_call') and v[1] > 0:
                e['mfma_busy_at_event_time'] = round(q['mfma_busy_cycles_per_call'] / (v[3] / n_k * 2.4e9 * 1024), 4)
        fam_out[k] = e
    roof = {'kernel': kind, 'bound': 'mfma', 'achieved': round(achieved, 2), 'peak': MFMA_PEAK_TFLOPS,
            'unit': 'TFLOP/s', 'frac': round(achieved / MFMA_PEAK_TFLOPS, 4), 'traffic': traffic,
            'traffic_unit': 'HBM bytes per launch (rocprofv3 PMC: FETCH_SIZE x2 + WRITE_SIZE, one pass each)',
            'traffic_source': traffic_src,
            # False: the PMC summary was taken with another build of libeegan_hip.so (stale figures)
            'traffic_matches_this_build': current if traffic_src else None,
            'traffic_git_head': (summ or {}).get('git_head'),
            'algorithmic_bytes_per_launch': round(nb / n),
            'algorithmic_flops_per_launch': round(fl / n),
            'pmc_over_algorithmic': round(traffic / (nb / n), 3) if traffic and nb > 0 else None,
            'launches_per_step': n // per, 'avg_launch_us': round(tsec / n * 1e6, 2),
            'timing': 'HIP start/stop events per dispatch (hipExtLaunchKernel) over %d eager step(s) of the same '
                      'workload right after the timed region' % per,
            'algorithmic_hbm_GBs': round(nb / tsec / 1e9, 1),
            'mfma_busy': pf.get('mfma_util') if pf.get('mfma_util_unit') else None,
            'mfma_busy_unit': pf.get('mfma_util_unit'),
            # the same counter (MFMA-busy cycles per launch, PMC pass) over THIS run's event-timed launch
            # duration x 2.4 GHz x 1024 SIMDs: the denominator `frac` uses, so the two compare directly
            # (counted cycles >= the FLOP count's cycles, so this is >= frac unless the counter under-counts)
            'mfma_busy_at_event_time': round(pf['mfma_busy_cycles_per_call'] / (tsec / n * 2.4e9 * 1024), 4)
            if pf.get('mfma_busy_cycles_per_call') and fl > 0 else None,
            # north_star's conv-path HBM figure: PMC FETCH+WRITE bytes over kernel time, / 8 TB/s
            # (wasted re-reads count as achieved bandwidth here; pmc_over_algorithmic says how many)
            'pmc_hbm_GBs': round(traffic / pf['avg_call_us'] / 1e3, 1) if traffic and pf.get('avg_call_us') else None,
            'pmc_hbm_frac': round(traffic / pf['avg_call_us'] / 1e3 / HBM_PEAK_GBS, 4)
            if traffic and pf.get('avg_call_us') else None,
            'conv_path_pmc_hbm_frac': conv_path_hbm_frac(pfams),
            'families': fam_out}
    # the same family in the replayed step (rocprofv3 kernel trace of the timed replays,
    # tools/rocprof_families.py): algorithmic FLOPs per step over in-step kernel time,
    # read from the summary so that it recomputes from that file alone
    if pf.get('frac_in_step') is not None:
        roof['frac_in_step'] = pf['frac_in_step']
        roof['in_step_ms_per_step'] = pf.get('ms_per_step')
        roof['in_step_avg_call_us'] = pf.get('avg_call_us')
        roof['pmc_over_algorithmic'] = pf.get('pmc_over_algorithmic', roof['pmc_over_algorithmic'])
        tp = (summ or {}).get('timing_pass', {}).get(kind)
        if tp:   # rocprof's view of the timing pass this line's `frac` comes from
            roof['rocprof_timing_pass_avg_call_us'] = tp['avg_call_us']
    cpath = (summ or {}).get('conv_path')
    if cpath:
        roof['conv_path_algorithmic_hbm_frac'] = cpath.get('algorithmic_hbm_frac')
        roof['conv_path_pmc_hbm_frac'] = cpath.get('pmc_hbm_frac', roof['conv_path_pmc_hbm_frac'])
        roof['conv_path_source'] = traffic_src
    out = {'metric': 'train images/sec at 256x256 CUB, G+D step', 'value': round(value, 3), 'unit': 'images/sec',
           'n_gpus': world, 'steps': args.steps, 'warmup': args.warmup, 'ms_per_step': round(ms, 3),
           'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None, 'dtype': 'bf16',
           'data': 'synthetic (U(-1,1) images, random captions/attributes/class ids), random-init weights',
           'config': {'workload': '%s full 3-stage 64->128->256 G+D step, GF=DF=%d, batch %d/GPU%s' % (
               CONFIGS[args.config][0], CONFIGS[args.config][1], B, ', class head %d' % ncls if ncls else ''),
               'model': 'EE-GAN Gen+ATTR_Enhance+Dis64/128/256+DAMSM(Inception-v3, biLSTM)',
               'global_batch': B * world, 'seq_len': 20, 'parallelism': 'dp%d' % world},
           'host_issue_ms_per_step': round(t_issue / args.steps * 1e3, 3),
           # host_issue: host time inside the timed loop (with replay pacing it includes the waits for the
           # previous replay); host_submit: one replay submitted with the GPU held busy (pure submission cost)
           'host_submit_ms_per_step': submit_ms,
           'replay_depth': StepGraph.DEPTH if use_graph else None,
           'execution': 'hip-graph replay of the captured step' if use_graph else 'eager',
           'roofline': roof}
    if timer is None:   # --no-timer: no dispatch was timed, so there is no roofline figure to report
        out['roofline'] = {'kernel': None, 'bound': 'mfma', 'achieved': None, 'peak': MFMA_PEAK_TFLOPS,
                           'unit': 'TFLOP/s', 'frac': None, 'traffic': None,
                           'note': 'not measured: --no-timer diagnostic run'}
    if args.config in CEILINGS:
        cm, ch = CEILINGS[args.config]
        out['step_roofline'] = {'img_s_per_gpu': round(value / world, 2), 'mfma_ceiling': cm, 'hbm_ceiling': ch,
                                'frac_of_bound': round(value / world / min(cm, ch), 4),
                                'source': 'BASELINE.md roofline ceilings per GPU'}
    if graph_error:
        out['graph_capture_error'] = graph_error
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            out['cpu_baseline'] = cpu_baseline_child(args.cpu_seconds)
        except Exception as e:  # baseline is reported, never fatal for the GPU measurement
            out['cpu_baseline'] = {'error': repr(e)}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()


if __name__ == '__main__':
    main()
