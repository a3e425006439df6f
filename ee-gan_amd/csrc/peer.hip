// One-shot peer-write all-reduce for the SyncBN statistics messages
// (reference: sync_batchnorm/batchnorm.py:90-111 -- the master gathers every
// device's (sum, ssum) pair, reduces and broadcasts the mean / inv-std back;
// here every rank reduces locally instead, so there is no master and no second
// hop).
//
// Each rank owns one small uncached "region" per stream lane, mapped into every
// peer's address space over IPC (xGMI on a multi-GPU node):
//
//   [0, 256)     flags[2][16] uint64   flags[parity][src] = epoch of src's slice
//   [256, 264)   counter uint64        epoch of the last completed call (local)
//   [264, 268)   error   uint32        set when a wait timed out (local)
//   [268, 272)   wait    uint32        the wait bound in seconds (0: 30 s); eegan_peer_set_wait
//   [512, ...)   data[2][16][cap] fp64 data[parity][src][i]
//
// A call (one 256-thread block): read epoch e = counter + 1, write this rank's
// message into slot [e & 1][rank] of EVERY rank's region (vector stores into
// peer memory), release-store flag[e & 1][rank] = e there, wait until all
// `world` flags of parity e & 1 in the OWN region equal e, then sum the slots
// in rank order 0..world-1 (identical bits on every rank), store counter = e.
// Double buffering by parity is safe: a rank reaches epoch e + 2 only after
// every peer finished epoch e + 1, i.e. after every peer finished reading the
// parity of epoch e.  The epoch lives on the device, so a captured call keeps
// counting when the step graph is replayed.
//
// Every wait is bounded (30 s of the 100 MHz wall clock by default, per region
// eegan_peer_set_wait / EEGAN_PEER_WAIT_S): a rank whose peer
// never arrives records an error and exits, so the grid always drains;
// eegan_peer_status reports it.  A call that finds the error word set in the
// own region or in any peer's (a wait of this lane already gave up on some
// rank) does not push or wait at all: it poisons its result at once, so after
// a dead peer only the first call of a lane pays the bound, not every later
// SyncBN call until the host's periodic check raises.
#include <string.h>

#include "common.h"
#include "../../include/eegan_hip.h"

namespace {

constexpr int PEER_MAXW = 16;
constexpr long OFF_CTR = 256, OFF_ERR = 264, OFF_WAIT = 268, OFF_DATA = 512;
// bounded wait for the peers' slices: long enough for host-side skew between
// ranks (a checkpoint save or an evaluation on one rank while the others wait
// in their next step), short enough that a dead peer ends the job: on timeout
// the error word is set and the result is poisoned with NaN (visible in the BN
// statistics at once); the trainer checks the error word and raises
// (eegan_hip.peer.PeerAllReduce.check, Trainer.check_collectives)
constexpr unsigned long long TICKS_PER_S = 100000000ull;  // wall_clock64: 100 MHz
constexpr unsigned DEFAULT_WAIT_S = 30;

struct PeerSet {
  char* base[PEER_MAXW];
};

EE_DEV unsigned long long* flag_at(char* base, int par, int src) {
  return reinterpret_cast<unsigned long long*>(base) + par * PEER_MAXW + src;
}
EE_DEV double* slot_at(char* base, int par, int src, int cap) {
  return reinterpret_cast<double*>(base + OFF_DATA) + ((long)par * PEER_MAXW + src) * cap;
}

__global__ __launch_bounds__(256) void peer_allreduce_kernel(double* t, int n, int cap, int rank, int world,
                                                             PeerSet ps) {
  const int tid = threadIdx.x;
  char* own = ps.base[rank];
  unsigned long long* ctr = reinterpret_cast<unsigned long long*>(own + OFF_CTR);
  __shared__ unsigned long long s_ep, s_wait;
  __shared__ int s_timeout;
  if (tid == 0) {
    s_ep = __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) + 1ull;
    unsigned err = 0;
    for (int p = 0; p < world; ++p)
      err |= __hip_atomic_load(reinterpret_cast<unsigned*>(ps.base[p] + OFF_ERR), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
    s_timeout = err != 0u;   // an earlier call of this lane gave up on a rank: poison at once
    const unsigned ws = __hip_atomic_load(reinterpret_cast<unsigned*>(own + OFF_WAIT), __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_SYSTEM);
    s_wait = (unsigned long long)(ws ? ws : DEFAULT_WAIT_S) * TICKS_PER_S;
  }
  __syncthreads();
  const unsigned long long ep = s_ep;
  const int par = (int)(ep & 1ull);
  const bool live = s_timeout == 0;
  const unsigned long long wait_ticks = s_wait;

  // push this rank's message into every rank's slot [par][rank]
  for (int p = 0; p < world && live; ++p) {
    double* dst = slot_at(ps.base[p], par, rank, cap);
    for (int i = tid; i < n; i += 256) dst[i] = t[i];
  }
  __threadfence_system();
  __syncthreads();
  if (tid < world && live)
    __hip_atomic_store(flag_at(ps.base[tid], par, rank), ep, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);

  // wait for every rank's slice in the own region (bounded)
  if (tid < world && live) {
    const unsigned long long t0 = wall_clock64();
    unsigned long long* f = flag_at(own, par, tid);
    while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != ep) {
      if (wall_clock64() - t0 > wait_ticks) {
        __hip_atomic_store(reinterpret_cast<unsigned*>(own + OFF_ERR), 1u + (unsigned)tid, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
        s_timeout = 1;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();

  // fixed-order combine: 0 + m_0 + m_1 + ... + m_{world-1}; NaN when a peer never arrived
  const bool poison = s_timeout != 0;
  for (int i = tid; i < n && poison; i += 256) t[i] = __builtin_nan("");
  for (int i = tid; i < n && !poison; i += 256) {
    double acc = 0.0;
    for (int q = 0; q < world; ++q) {
      const unsigned long long* src = reinterpret_cast<const unsigned long long*>(slot_at(own, par, q, cap)) + i;
      acc += __longlong_as_double((long long)__hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
    }
    t[i] = acc;
  }
  __syncthreads();
  if (tid == 0) __hip_atomic_store(ctr, ep, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

}  // namespace

extern "C" {

long eegan_peer_region_bytes(int cap) {
  if (cap < 1) return -1;
  return OFF_DATA + 2L * PEER_MAXW * cap * (long)sizeof(double);
}

int eegan_peer_alloc(long bytes, void** base, void* handle) {
  if (bytes < OFF_DATA || !base || !handle) {
    ee_set_error("peer_alloc: bad arguments (bytes=%ld)", bytes);
    return -1;
  }
  void* p = nullptr;
  hipError_t e = hipExtMallocWithFlags(&p, (size_t)bytes, hipDeviceMallocUncached);
  if (e != hipSuccess) {
    ee_set_error("peer_alloc: hipExtMallocWithFlags(uncached, %ld): %s", bytes, hipGetErrorString(e));
    return -1;
  }
  e = hipMemset(p, 0, (size_t)bytes);
  if (e == hipSuccess) e = hipDeviceSynchronize();
  hipIpcMemHandle_t h;
  if (e == hipSuccess) e = hipIpcGetMemHandle(&h, p);
  if (e != hipSuccess) {
    (void)hipFree(p);
    ee_set_error("peer_alloc: %s", hipGetErrorString(e));
    return -1;
  }
  memcpy(handle, &h, sizeof(h));
  *base = p;
  return 0;
}

int eegan_peer_open(const void* handle, void** base) {
  hipIpcMemHandle_t h;
  memcpy(&h, handle, sizeof(h));
  hipError_t e = hipIpcOpenMemHandle(base, h, hipIpcMemLazyEnablePeerAccess);
  if (e != hipSuccess) {
    ee_set_error("peer_open: hipIpcOpenMemHandle: %s", hipGetErrorString(e));
    return -1;
  }
  return 0;
}

int eegan_peer_close(void* base) {
  hipError_t e = hipIpcCloseMemHandle(base);
  if (e != hipSuccess) {
    ee_set_error("peer_close: %s", hipGetErrorString(e));
    return -1;
  }
  return 0;
}

int eegan_peer_free(void* base) {
  hipError_t e = hipFree(base);
  if (e != hipSuccess) {
    ee_set_error("peer_free: %s", hipGetErrorString(e));
    return -1;
  }
  return 0;
}

int eegan_peer_allreduce_f64(double* t, int n, int cap, int rank, int world, void* const* bases, hipStream_t s) {
  if (world < 1 || world > PEER_MAXW || rank < 0 || rank >= world || n < 0 || n > cap || !bases) {
    ee_set_error("peer_allreduce: bad arguments (n=%d cap=%d rank=%d world=%d, at most %d ranks)", n, cap, rank,
                 world, PEER_MAXW);
    return -1;
  }
  PeerSet ps = {};
  for (int p = 0; p < world; ++p) {
    if (!bases[p]) {
      ee_set_error("peer_allreduce: region of rank %d not mapped", p);
      return -1;
    }
    ps.base[p] = static_cast<char*>(bases[p]);
  }
  ee_launch(peer_allreduce_kernel, dim3(1), dim3(256), 0, s, t, n, cap, rank, world, ps);
  EE_LAUNCH_CHECK("peer_allreduce_kernel");
}

int eegan_peer_set_wait(void* own, int seconds) {
  if (!own || seconds < 1 || seconds > 86400) {
    ee_set_error("peer_set_wait: bad arguments (seconds=%d, 1..86400)", seconds);
    return -1;
  }
  const unsigned v = (unsigned)seconds;
  hipError_t e = hipMemcpy(static_cast<char*>(own) + OFF_WAIT, &v, sizeof(v), hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    ee_set_error("peer_set_wait: %s", hipGetErrorString(e));
    return -1;
  }
  return 0;
}

int eegan_peer_status(void* own, int reset, int* timed_out) {
  unsigned err = 0;
  hipError_t e = hipMemcpy(&err, static_cast<char*>(own) + OFF_ERR, sizeof(err), hipMemcpyDeviceToHost);
  if (e == hipSuccess && reset && err) e = hipMemset(static_cast<char*>(own) + OFF_ERR, 0, sizeof(err));
  if (e != hipSuccess) {
    ee_set_error("peer_status: %s", hipGetErrorString(e));
    return -1;
  }
  *timed_out = (int)err;
  return 0;
}

}  // extern "C"
