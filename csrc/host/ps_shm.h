// CPU parameter server over a shared-memory data plane (parallel/ps.py, transport "shm").
//
// The reference's parameter servers are CPU tasks (tf.train.replica_device_setter places
// the variables on /job:ps, /root/reference/main.py:80-82) that apply each worker's
// gradients as they arrive (mnist_input.py:261-264).  On one MI355X node the GPUs belong
// to the workers: a PS that launches its optimizer on a GPU time-slices that GPU with the
// workers' step graphs (profiles/r3/ps/: a co-located worker's 78 us step stretched to
// 0.28-0.62 ms).  Here the PS keeps its shard's fp32 master / momentum / EMA in host
// memory and serves pushes from a shared-memory segment with this native loop:
//
//   worker: DMA its gradient slice into its push slot (the slot is pinned with
//           hipHostRegister), write the int64 sequence stamp, publish push_seq;
//   PS:     sees push_seq change, checks the stamp, applies the optimizer (exact IEEE
//           per element: bitwise runtime/torchnet.torch_update), copies the parameters
//           into the worker's reply slot, publishes reply_seq (+ global step / stop);
//   worker: spins on reply_seq, DMAs the reply into its device parameters.
//
// No GPU work, no Python and no control-plane message per update.  Control messages
// (HELLO / STATE / DONE / RESET) still travel on the gloo group: a worker raises its
// pending flag first, and the loop returns to Python to receive it.
//
// Segment layout (bytes; mirrored by parallel/ps.py ShmLayout): a 4096-byte header page (so every
// worker block starts on a page: a worker pins -- hipHostRegister -- only its own block), then
// one block per worker at wblock stride: control words int64[16] at ctrl_off, the push
// slot (slot_floats floats, the last 8 bytes = the stamp) at push_off, the reply
// parameters at reply_off.
#pragma once
#include <math.h>
#include <stdint.h>
#include <string.h>
#include <time.h>

#include <algorithm>
#include <thread>
#include <vector>

namespace mnistx_host {

constexpr int64_t kPsHdr = 4096;   // header page (ShmLayout.HDR)
enum PsCtrl { C_PUSH_SEQ = 0, C_PENDING = 1, C_REPLY_SEQ = 2, C_REPLY_GSTEP = 3, C_REPLY_STOP = 4, C_REPLY_APPLIED = 5 };
enum PsServeRc { PS_CTRL = 0, PS_BAD_STAMP = 1, PS_KILL = 2, PS_IDLE_TIMEOUT = 3 };

struct PsLayout {
  int64_t n, W, slot_floats, wblock, ctrl_off, push_off, reply_off;
};

struct PsOpt {
  double lr0, decay_rate;
  int64_t decay_steps;
  double momentum;
  int nesterov, use_momentum;
  double ema_max;   // < 0: no EMA
};

struct PsState {   // persists across ps_serve calls (Python owns the arrays)
  int64_t gstep, max_steps, applied, rejected, kill_step;
  int64_t* per_worker;     // [W]
  int64_t* last_seq;       // [W]: the last push sequence served per worker
  int32_t* arrivals;       // [arrivals_cap]: worker of every applied push, in order
  int64_t arrivals_cap, narr;
  const int64_t* mark_steps;
  double* mark_times;      // CLOCK_MONOTONIC seconds (time.perf_counter's clock)
  int nmarks;
  double phase[3];         // idle / apply / reply seconds
  int last;                // round-robin cursor
  double idle_timeout;     // seconds without any push or control flag -> PS_IDLE_TIMEOUT
};

inline double ps_now() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

template <bool MOM, bool NEST, bool EMA>
inline void ps_apply_k(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                       float* __restrict__ e, const float* __restrict__ wd, int64_t n, float lr, float mu, float omd) {
  const float one = 1.0f;
  for (int64_t i = 0; i < n; ++i) {
    const float pi = p[i];
    const float gi = g[i] * one + wd[i] * pi;
    float u = gi;
    if constexpr (MOM) {
      const float mi = m[i] * mu + gi;
      m[i] = mi;
      u = NEST ? gi + mu * mi : mi;
    }
    const float pn = pi - lr * u;
    p[i] = pn;
    if constexpr (EMA) e[i] = e[i] - omd * (e[i] - pn);
  }
}
// the same loops built for AVX2 (8 lanes; still no FMA) where the CPU has it
template <bool MOM, bool NEST, bool EMA>
__attribute__((target("avx2"))) void ps_apply_avx2(float* __restrict__ p, const float* __restrict__ g,
                                                  float* __restrict__ m, float* __restrict__ e,
                                                  const float* __restrict__ wd, int64_t n, float lr, float mu,
                                                  float omd) {
  const float one = 1.0f;
  for (int64_t i = 0; i < n; ++i) {
    const float pi = p[i];
    const float gi = g[i] * one + wd[i] * pi;
    float u = gi;
    if constexpr (MOM) {
      const float mi = m[i] * mu + gi;
      m[i] = mi;
      u = NEST ? gi + mu * mi : mi;
    }
    const float pn = pi - lr * u;
    p[i] = pn;
    if constexpr (EMA) e[i] = e[i] - omd * (e[i] - pn);
  }
}

// element-wise, so any split of [0, n) gives the same bits: shards of >= 1M parameters (the
// reference CNN's 3.46M: ~9 ms on one core, memory bound) run on up to 8 threads
template <bool MOM, bool NEST, bool EMA>
inline void ps_apply_dispatch(float* p, const float* g, float* m, float* e, const float* wd, int64_t n, float lr,
                              float mu, float omd) {
  static const bool avx2 = __builtin_cpu_supports("avx2");
  auto run = [&](int64_t a, int64_t b) {
    if (avx2) ps_apply_avx2<MOM, NEST, EMA>(p + a, g + a, m + a, e + a, wd + a, b - a, lr, mu, omd);
    else ps_apply_k<MOM, NEST, EMA>(p + a, g + a, m + a, e + a, wd + a, b - a, lr, mu, omd);
  };
  const int64_t T = n >= (1 << 20) ? std::min<int64_t>(8, std::max(1u, std::thread::hardware_concurrency())) : 1;
  if (T <= 1) {
    run(0, n);
    return;
  }
  const int64_t chunk = (n + T - 1) / T / 16 * 16 + 16;
  std::vector<std::thread> th;
  for (int64_t a = chunk; a < n; a += chunk) th.emplace_back(run, a, std::min(n, a + chunk));
  run(0, std::min(n, chunk));
  for (auto& t : th) t.join();
}

// The K9 update of one shard, element by element with the rounding of
// runtime/torchnet.torch_update (separate IEEE ops, no contraction: the host build compiles
// ISO C++ -- -ffp-contract=off -- and the AVX2 variant has no FMA):
//   g = grads * 1 + wd * p;  m = m * mu + g;  u = nesterov ? g + mu * m : m;  p -= lr * u;
//   ema -= (1 - d) * (ema - p),  d = min(ema_max, (1 + step) / (10 + step)).
inline void ps_apply(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                     float* __restrict__ e, const float* __restrict__ wd, int64_t n, const PsOpt& o, int64_t step) {
  double lrd = o.lr0;
  if (o.decay_steps > 0) lrd = o.lr0 * pow(o.decay_rate, (double)(step / o.decay_steps));
  const float lr = (float)lrd, mu = (float)o.momentum;
  const bool ema = o.ema_max >= 0.0;
  double d = (1.0 + (double)step) / (10.0 + (double)step);
  if (ema && d > o.ema_max) d = o.ema_max;
  const float omd = (float)(1.0 - d);
  const int code = (o.use_momentum ? 4 : 0) | (o.use_momentum && o.nesterov ? 2 : 0) | (ema ? 1 : 0);
  switch (code) {
    case 0: ps_apply_dispatch<false, false, false>(p, g, m, e, wd, n, lr, mu, omd); break;
    case 1: ps_apply_dispatch<false, false, true>(p, g, m, e, wd, n, lr, mu, omd); break;
    case 4: ps_apply_dispatch<true, false, false>(p, g, m, e, wd, n, lr, mu, omd); break;
    case 5: ps_apply_dispatch<true, false, true>(p, g, m, e, wd, n, lr, mu, omd); break;
    case 6: ps_apply_dispatch<true, true, false>(p, g, m, e, wd, n, lr, mu, omd); break;
    default: ps_apply_dispatch<true, true, true>(p, g, m, e, wd, n, lr, mu, omd); break;
  }
}

inline volatile int64_t* ps_ctrl(uint8_t* base, const PsLayout& L, int64_t w) {
  return (volatile int64_t*)(base + kPsHdr + w * L.wblock + L.ctrl_off);
}

// Serve pushes until a worker raises its control flag (PS_CTRL), a push carries a stamp
// other than its announced sequence (PS_BAD_STAMP: never applied), the fault-injection
// kill step is reached (PS_KILL) or nothing happens for idle_timeout seconds.  *who = the
// worker concerned.  Workers are served round-robin from the last one served (each
// worker has at most one push in flight, so none waits behind another twice).
inline int ps_serve(uint8_t* base, const PsLayout& L, float* params, float* mom, float* ema, const float* wd,
                    const PsOpt& o, PsState& S, int* who) {
  double t_idle = ps_now(), t_last_event = t_idle;
  uint32_t spins = 0;
  for (;;) {
    for (int64_t w = 0; w < L.W; ++w)
      if (__atomic_load_n(ps_ctrl(base, L, w) + C_PENDING, __ATOMIC_ACQUIRE) != 0) {
        S.phase[0] += ps_now() - t_idle;
        *who = (int)w;
        return PS_CTRL;
      }
    int found = -1;
    int64_t seq = 0;
    for (int64_t k = 1; k <= L.W; ++k) {
      const int64_t w = (S.last + k) % L.W;
      const int64_t s = __atomic_load_n(ps_ctrl(base, L, w) + C_PUSH_SEQ, __ATOMIC_ACQUIRE);
      if (s != S.last_seq[w]) {
        found = (int)w;
        seq = s;
        break;
      }
    }
    if (found < 0) {
      if (++spins > 2000) {   // ~tens of us of pure spinning: yield the core between polls
        const double t = ps_now();
        if (t - t_last_event > S.idle_timeout) {
          S.phase[0] += t - t_idle;
          *who = -1;
          return PS_IDLE_TIMEOUT;
        }
        timespec ts{0, 20000};
        nanosleep(&ts, nullptr);
      } else {
        __builtin_ia32_pause();
      }
      continue;
    }
    spins = 0;
    double t = ps_now();
    S.phase[0] += t - t_idle;
    const int w = found;
    S.last = w;
    S.last_seq[w] = seq;
    uint8_t* blk = base + kPsHdr + (int64_t)w * L.wblock;
    const float* g = (const float*)(blk + L.push_off);
    int64_t stamp;
    memcpy(&stamp, (const uint8_t*)g + L.slot_floats * 4 - 8, 8);
    if (stamp != seq) {
      *who = w;
      return PS_BAD_STAMP;
    }
    if (S.gstep < S.max_steps) {
      ps_apply(params, g, mom, ema, wd, L.n, o, S.gstep);
      S.gstep += 1;
      S.applied += 1;
      S.per_worker[w] += 1;
      if (S.narr < S.arrivals_cap) S.arrivals[S.narr++] = w;
    } else {
      S.rejected += 1;   // in flight past the stop point: answered, not applied
    }
    double t2 = ps_now();
    S.phase[1] += t2 - t;
    memcpy(blk + L.reply_off, params, (size_t)L.n * 4);
    volatile int64_t* c = ps_ctrl(base, L, w);
    c[C_REPLY_GSTEP] = S.gstep;
    c[C_REPLY_STOP] = S.gstep >= S.max_steps ? 1 : 0;
    c[C_REPLY_APPLIED] = S.applied;
    __atomic_store_n(c + C_REPLY_SEQ, seq, __ATOMIC_RELEASE);
    t = ps_now();
    S.phase[2] += t - t2;
    for (int i = 0; i < S.nmarks; ++i)
      if (S.gstep == S.mark_steps[i] && S.mark_times[i] == 0.0) S.mark_times[i] = t;
    t_idle = t_last_event = t;
    if (S.kill_step > 0 && S.gstep >= S.kill_step) {
      *who = w;
      return PS_KILL;
    }
  }
}

}  // namespace mnistx_host
