"""One process per GPU under an UNCHANGED reference train.py.

The reference trains data-parallel inside ONE process: `train.py:513` sets
CUDA_VISIBLE_DEVICES = args.gpu_ids, `train.py:220-228` wraps G / ATTR_Enhance
/ the D's in (SyncBN-aware) nn.DataParallel, and train.py never creates a
process group.  Launched as one process per GPU (torchrun), nothing in that
file pins a rank to its GPU or joins the ranks.  This module does both when
the drop-in package is imported -- `train.py:22-29` imports it long before
line 513 and before anything touches the GPU:

  * pin_rank_device(): the rank's GPU becomes the only one the HIP runtime will
    enumerate (ROCR_VISIBLE_DEVICES = that GPU, HIP_VISIBLE_DEVICES = 0; the HIP
    runtime and torch both give HIP_VISIBLE_DEVICES priority over the
    CUDA_VISIBLE_DEVICES that train.py:513 writes later), so torch.device('cuda')
    (train.py:114) is the rank's GPU and nn.DataParallel sees one device and
    stays a pass-through;
  * init_process_group(): joins the ranks from torchrun's env (RANK,
    WORLD_SIZE, MASTER_ADDR, MASTER_PORT); backend EEGAN_DIST_BACKEND, else
    "nccl" (RCCL) when a GPU is visible, "gloo" otherwise.

Both run only when torchrun's env says WORLD_SIZE > 1 (LOCAL_RANK and
LOCAL_WORLD_SIZE present), at most once per process, never in a
multiprocessing child of a rank (train.py's DataLoader workers, started with
'spawn' at train.py:35, re-import train.py's modules with the rank's env), and
never touch the GPU themselves (device counting goes through amdsmi or the
visible-device variables, not the HIP runtime).  EEGAN_AUTO_DIST=0 turns both
off for callers that set devices and start the process group themselves
(bench.py, eegan_hip.dist.init_from_env users).

The reference's DataParallel SCATTERS one batch over its GPUs
(train.py:220-228); one process per GPU instead runs train.py once per rank
with the same seed (train.py:521-525), the same shuffled DataLoader
(train.py:277-278) and the same noise draws (train.py:189).  data_shard()
gives the drop-in TextDataset its rank-strided shard, and offset_rank_rngs()
(called by that constructor, i.e. after train.py has seeded) moves every rank
but rank 0 onto its own torch / numpy / python random streams, so each rank
draws its own captions, crops and noise.  Model weights initialised from the
offset streams differ across ranks; eegan_hip.dist.ensure_grad_hooks
broadcasts rank 0's parameters and buffers at the first forward, as DDP does
at construction.
"""
import os

_STATE = {'pinned': None, 'pg': False, 'rng_offset': None}


def _mp_child():
    """True in a multiprocessing child (DataLoader worker, pool process) --
    also while a 'spawn' / 'forkserver' child is still importing the parent's
    main module (multiprocessing.spawn.prepare), before parent_process() is
    set: that is exactly when train.py's imports reach this module."""
    import sys
    import multiprocessing
    return (multiprocessing.parent_process() is not None or '--multiprocessing-fork' in sys.argv
            or bool(getattr(multiprocessing.current_process(), '_inheriting', False)))


def torchrun_world():
    """WORLD_SIZE of a torchrun-launched process (1 otherwise)."""
    if 'LOCAL_RANK' not in os.environ or 'LOCAL_WORLD_SIZE' not in os.environ:
        return 1
    try:
        return int(os.environ.get('WORLD_SIZE', '1'))
    except ValueError:
        return 1


def auto_enabled():
    return os.environ.get('EEGAN_AUTO_DIST', '1') != '0' and torchrun_world() > 1


def _visible_physical(n):
    """The devices the runtime would enumerate now, as ROCR-level ids
    (indices into the ROCr device list, or UUID strings)."""
    rocr = os.environ.get('ROCR_VISIBLE_DEVICES')
    base = [t.strip() for t in rocr.split(',') if t.strip()] if rocr else None
    sel = os.environ.get('HIP_VISIBLE_DEVICES') or os.environ.get('CUDA_VISIBLE_DEVICES')
    if sel:
        toks = [t.strip() for t in sel.split(',') if t.strip()]
        if base is not None:
            out = []
            for t in toks:
                if not t.isdigit() or int(t) >= len(base):
                    break   # the runtime stops at the first invalid ordinal
                out.append(base[int(t)])
            return out[:n]
        return toks[:n]
    if base is not None:
        return base[:n]
    return [str(i) for i in range(n)]


def _env_uuid_devices():
    """True when a visible-device variable names devices by UUID: torch's
    device count then falls back to hipGetDeviceCount, which starts the HIP
    runtime before the pin could take effect."""
    for k in ('ROCR_VISIBLE_DEVICES', 'HIP_VISIBLE_DEVICES', 'CUDA_VISIBLE_DEVICES'):
        v = os.environ.get(k)
        if v and any(t.strip() and not t.strip().isdigit() for t in v.split(',')):
            return True
    return False


def _device_count():
    """Devices the runtime would enumerate, without starting it."""
    if _env_uuid_devices():
        return len(_visible_physical(1 << 16))
    import torch
    return torch.cuda.device_count()   # amdsmi on this build: no HIP runtime init


def pin_rank_device():
    """Make LOCAL_RANK's GPU the process's only visible device (before the HIP
    runtime starts).  Several ranks per GPU (more ranks than GPUs) share
    round-robin.  Returns the ROCR-level id pinned ('set_device:<i>' when the
    runtime was already up and the rank's device was selected instead), or
    None when nothing is visible."""
    if _STATE['pinned'] is not None or not auto_enabled():
        return _STATE['pinned']
    import torch
    local = int(os.environ['LOCAL_RANK'])
    if torch.cuda.is_initialized():
        # too late for the environment: select the rank's device in the running runtime
        n = torch.cuda.device_count()
        if n <= 0:
            raise RuntimeError('eegan_hip: rank %d has no visible GPU' % local)
        torch.cuda.set_device(local % n)
        _STATE['pinned'] = 'set_device:%d' % (local % n)
        return _STATE['pinned']
    n = _device_count()
    if n <= 0:
        return None
    phys = _visible_physical(n)
    if not phys:
        return None
    mine = phys[local % len(phys)]
    os.environ['ROCR_VISIBLE_DEVICES'] = mine
    os.environ['HIP_VISIBLE_DEVICES'] = '0'
    os.environ.pop('CUDA_VISIBLE_DEVICES', None)
    _STATE['pinned'] = mine
    return mine


def init_process_group():
    """Join the torchrun ranks (no-op when a group exists or auto mode is off)."""
    if not auto_enabled():
        return False
    import torch.distributed as dist
    if not dist.is_available() or dist.is_initialized():
        return dist.is_available() and dist.is_initialized()
    backend = os.environ.get('EEGAN_DIST_BACKEND')
    if not backend:
        import torch
        backend = 'nccl' if torch.cuda.device_count() > 0 else 'gloo'
    os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
    dist.init_process_group(backend=backend)
    _STATE['pg'] = True
    import atexit

    def _close():
        try:
            if dist.is_initialized():
                dist.destroy_process_group()
        except Exception:   # interpreter shutdown: best effort
            pass
    atexit.register(_close)
    return True


def setup():
    """Import-time entry (eegan_hip/__init__): pin, then join -- in the rank
    process itself, not in its DataLoader workers."""
    if _mp_child():
        return
    pin_rank_device()
    init_process_group()


def data_shard():
    """(rank, world) of the data-parallel job the drop-in dataset shards over:
    the process group's when one is up with more than one rank, else (0, 1)."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def offset_rank_rngs(rank):
    """Put rank `rank` (> 0) on random streams of its own: torch's (CPU and
    every device), numpy's global RandomState and python's `random`, each
    re-seeded from a function of its current state and the rank.  All ranks
    hold identical states here (train.py:521-525 seeded them alike), so the
    new streams differ across ranks and are reproducible; rank 0 keeps the
    reference's streams.  Once per process."""
    if rank <= 0 or _STATE['rng_offset'] is not None:
        return
    import random
    import numpy as np
    import torch
    mix = 0x9E3779B97F4A7C15 * rank
    tseed = (torch.initial_seed() ^ mix) % (1 << 63)
    torch.manual_seed(tseed)
    key0 = int(np.random.get_state()[1][0])
    np.random.seed((key0 ^ mix) & 0xFFFFFFFF)
    random.seed(random.getrandbits(64) ^ mix)
    _STATE['rng_offset'] = rank


def check_process_group():
    """Raise when torchrun launched several ranks but no process group joins
    them: the ranks would otherwise train N unsynchronised copies."""
    if torchrun_world() <= 1:
        return
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        return
    raise RuntimeError(
        'eegan_hip: launched as rank %s of WORLD_SIZE=%d but no torch.distributed process group exists; the '
        'drop-in modules start one at import unless EEGAN_AUTO_DIST=0 -- then call eegan_hip.dist.init_from_env() '
        '(or torch.distributed.init_process_group) before the first forward'
        % (os.environ.get('RANK', '?'), torchrun_world()))
