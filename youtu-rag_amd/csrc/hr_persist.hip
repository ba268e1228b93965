// hr_persist.hip -- the persistent FILTER: one long-lived launch streams the corpus for consecutive batches.
//
// A pipelined shard pays each FILTER launch's ramp and tail -- waves of one launch end tens of microseconds apart,
// and the next launch's workgroups only take a CU once the previous one frees it (the 1.25M-row step at
// 0.75 of 8 TB/s, against 0.86 for one 10M launch).  Here an INSTANCE of k_scan_persist (one workgroup per CU on the
// CUs the tail stream leaves free) runs batch after batch: a workgroup that is through its share of batch e's tiles
// restages batch e+1's queries into its LDS and goes on, so the chip keeps reading while the last tiles of batch e
// finish elsewhere -- the stream is as continuous as one long launch (device stamps: a workgroup starts batch e+1
// within ~1 us of finishing batch e; every workgroup's start and end spread over ~23 us).
// Measured ("Persistent FILTER"): faster than per-batch launches for 4.2M-5.1M-row shards (5M rows:
// 1.53 vs 1.58 ms/step), not below, where the dual FILTER streams already overlap consecutive launches -- so the
// default (mode 1) takes it in that range only.
//
// Hand-offs (all inside one device; MI355X_MICROARCH.md "inter-workgroup visibility" / cdna_hip_programming.md
// Guideline 16 -- agent-scope atomics on the control words, a release before every signal, one acquire after every
// admission):
//  * host -> instance: the batch's query prep + SAMPLE run on the index's pre stream as before; a one-lane kernel
//    behind them (k_persist_post) raises `posted` and ADMITS the batch to the running instance with one
//    compare-and-swap of `gate` (admitted-through epoch, bit 31 = closed).  The workgroups poll `gate` (one lane,
//    relaxed, s_sleep between polls) and take the admission with one agent-scope acquire before reading the batch's
//    query fragments and floors with plain loads;
//  * idle exit: when no batch is admitted for idle_ticks of s_memrealtime (100 MHz), workgroup 0's leader closes
//    the gate with a compare-and-swap -- the CAS decides between "admitted" and "closed" for that epoch once, for
//    every workgroup -- and the instance exits.  A batch whose CAS then fails is not lost: an instance is launched
//    behind every batch on the persist stream, gated by that batch's post event; it starts after the running instance
//    has exited, finds from `next_epoch` whether its batch was processed, and processes it (and the batches admitted
//    after it) if not -- otherwise it exits at once;
//  * instance -> tail: each workgroup, through a batch, drains its write-through (sc1) candidate and count stores
//    and adds 1 to the slot's `done` counter; a one-lane kernel on the tail stream (k_persist_wait) polls it up to the batch's target
//    and the tail's select / rescore follow it in stream order (a kernel boundary: their own acquire).
// Every wait is bounded (an exit condition every wave reaches): the instance's non-leader polls give up after
// kHardTicks, the tail wait after kHardTicks too; either sets `error` (and the host's pinned error word) instead of
// hanging the GPU.
#include "hr_internal.hpp"
#include "hr_kernels.hpp"

namespace hr {

namespace {

constexpr uint32_t kGateClosed = 0x80000000u;
constexpr uint64_t kHardTicks = 200000000ull;  // 2 s of s_memrealtime (100 MHz): a wait this long is a failure

__device__ __forceinline__ uint32_t ld_agent(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(uint32_t* p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void report_error(PersistCtl* c, uint32_t* host_err, uint32_t code) {
    st_agent(&c->error, code);
    if (host_err) __hip_atomic_store(host_err, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// one lane: wait until epoch e is admitted (1) or the gate closed before it (0)
__device__ uint32_t wait_admission(PersistCtl* c, uint32_t e, bool leader, uint32_t idle_ticks, uint32_t* host_err) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        const uint32_t g = ld_agent(&c->gate);
        if ((g & ~kGateClosed) >= e) {
            // ONE agent acquire after the match: the batch's query fragments / floors are then read with plain loads
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            return 1u;
        }
        if (g & kGateClosed) return 0u;
        const uint64_t dt = __builtin_amdgcn_s_memrealtime() - t0;
        if (leader && dt > idle_ticks) {
            uint32_t expect = e - 1;  // (open and not admitting e: admitted through exactly e - 1)
            if (__hip_atomic_compare_exchange_strong(&c->gate, &expect, expect | kGateClosed, __ATOMIC_RELAXED,
                                                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
                return 0u;
            continue;  // admitted meanwhile
        }
        if (dt > kHardTicks) {
            report_error(c, host_err, 1u);
            return 0u;
        }
        __builtin_amdgcn_s_sleep(2);
    }
}

// one lane, once per workgroup: wait until this instance's leader has opened the gate (opened >= e0; epochs only grow)
__device__ uint32_t wait_opened(PersistCtl* c, uint32_t e0, uint32_t* host_err) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(&c->opened, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < e0) {
        if (__builtin_amdgcn_s_memrealtime() - t0 > kHardTicks) {
            report_error(c, host_err, 1u);
            return 0u;
        }
        __builtin_amdgcn_s_sleep(2);
    }
    return 1u;
}

// The instance.  pa.e0: the epoch it was launched for (its post has completed: the launch waited for its event).
template <int MT, int DT, int P>
__global__ __launch_bounds__(kScanThreads, 2) void k_scan_persist(PersistLaunch pa) {
    __shared__ uint32_t cmd;
    PersistCtl* const c = pa.ctl;
    const int tid = threadIdx.x;
    const bool leader = blockIdx.x == 0 && tid == 0;
    bool first_wait = true;  // (tid 0) the next admission poll is this workgroup's first
    uint32_t e = pa.e0;
    if (tid == 0) cmd = ld_agent(&c->next_epoch) > e ? 0u : 1u;  // processed by an earlier instance: nothing to do
    __syncthreads();
    if (!cmd) return;
    if (leader) {
        __hip_atomic_fetch_add(&c->runs, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // open the gate for this instance: every batch posted so far is ready (its post followed its SAMPLE); with a
        // close requested (quiesce), keep it closed -- this instance then serves its own batch only.  A CAS loop, not
        // a store: a k_persist_post admitting a batch between the read of `posted` and the write would otherwise be
        // overwritten (that epoch then waited for the idle exit)
        uint32_t g = ld_agent(&c->gate);
        for (;;) {
            const uint32_t p = ld_agent(&c->posted);
            const uint32_t want = ld_agent(&c->stop) ? ((e - 1) | kGateClosed) : (p > e ? p : e);
            if (__hip_atomic_compare_exchange_strong(&c->gate, &g, want, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT))
                break;
        }
        // the other workgroups wait for this before their first admission poll (they could otherwise read the previous
        // instance's closed gate and exit after e0)
        __hip_atomic_store(&c->opened, e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
    for (bool first = true;; first = false) {
        const int s = (int)((e - 1) % kPersistSlots);
        if (!first) {
            if (tid == 0) {
                cmd = 1u;
                if (first_wait && !leader) cmd = wait_opened(c, pa.e0, pa.host_err);
                first_wait = false;
                if (cmd) cmd = wait_admission(c, e, leader, pa.idle_ticks, pa.host_err);
            }
            __syncthreads();
            if (!cmd) break;
        }
        if (tid == 0) {
            const unsigned long long t = __builtin_amdgcn_s_memrealtime();
            __hip_atomic_fetch_min(&c->t_start0[e % kPersistRing], t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_max(&c->t_start1[e % kPersistRing], t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        {
            ScanArgs a = pa.a;
            auto at = [&](auto* p, int64_t stride) { return (decltype(p))((uintptr_t)p + (uintptr_t)(s * stride)); };
            a.qfrag = at(a.qfrag, pa.st_qfrag);
            a.mkeys = at(a.mkeys, pa.st_mkeys);
            a.floor_q = at(a.floor_q, pa.st_floor);
            a.pbuf = at(a.pbuf, pa.st_pbuf);
            a.pcnt = at(a.pcnt, pa.st_pcnt);
            a.dyn_q = at(a.dyn_q, pa.st_dynq);
            scan_body<MT, DT, 2, P, SCAN_FILTER, true, kScanThreads, true>(a);
        }
        // through batch e: the lean body stores its candidates and counts write-through (sc1, Guideline 16 R1), so
        // every wave drains them, the workgroup meets, and one lane adds the slot's arrival -- no release fence
        // (an L2 writeback per workgroup per batch: 28 per XCD every batch)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) {
            __hip_atomic_fetch_add(&c->arr[e % kPersistRing], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const unsigned long long t = __builtin_amdgcn_s_memrealtime();
            __hip_atomic_fetch_max(&c->t_end[e % kPersistRing], t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_min(&c->t_end0[e % kPersistRing], t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        ++e;
    }
    if (leader) st_agent(&c->next_epoch, e);
}

// behind batch e's query prep + SAMPLE on the pre stream: batch e is ready; admit it to a running instance
__global__ void k_persist_post(PersistCtl* c, uint32_t e) {
    if (threadIdx.x == 0) {
        const int r = (int)(e % kPersistRing);  // the epoch's stamps (its previous use, e - ring, is long through)
        c->t_end[r] = 0ull;
        c->t_start1[r] = 0ull;
        c->t_start0[r] = ~0ull;
        c->t_end0[r] = ~0ull;
        c->arr[r] = (unsigned long long)e << 32;  // no arrival yet (published by the release below)
        c->t_post[r] = __builtin_amdgcn_s_memrealtime();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        __hip_atomic_fetch_max(&c->posted, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        uint32_t expect = e - 1;
        __hip_atomic_compare_exchange_strong(&c->gate, &expect, e, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
    }
}

// quiesce (pre stream, behind every post): close the gate; the running instance exits once it is through the
// batches admitted so far, and later instances serve only their own batch
__global__ void k_persist_close(PersistCtl* c) {
    if (threadIdx.x == 0) {
        st_agent(&c->stop, 1u);
        __hip_atomic_fetch_or(&c->gate, kGateClosed, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// tail stream: wait until all nwg workgroups are through epoch e (its arrival word carries e's tag and nwg arrivals);
// a wait that gives up marks the slot's batch failed (slot_fail[s], read by the k_select behind it: the batch goes to
// the exact collect pass)
__global__ void k_persist_wait(PersistCtl* c, uint32_t e, uint32_t nwg, uint32_t* host_err) {
    if (threadIdx.x != 0) return;
    const int s = (int)((e - 1) % kPersistSlots);
    const unsigned long long want = ((unsigned long long)e << 32) | nwg;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        const unsigned long long v =
            __hip_atomic_load(&c->arr[e % kPersistRing], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((v >> 32) == e && v >= want) break;
        if (__builtin_amdgcn_s_memrealtime() - t0 > kHardTicks) {
            report_error(c, host_err, 2u);
            st_agent(&c->slot_fail[s], 1u);
            return;
        }
        __builtin_amdgcn_s_sleep(2);
    }
    st_agent(&c->slot_fail[s], 0u);
}

template <int MT, int DT, int P>
int launch_t(int cus, const PersistLaunch& pa, int lds, hipStream_t st) {
    auto kern = k_scan_persist<MT, DT, P>;
    static bool attr[64] = {};
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev));
    if (!attr[dev & 63]) {
        HIP_TRY(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024 - 64));
        attr[dev & 63] = true;
    }
    hipLaunchKernelGGL(kern, dim3((unsigned)cus), dim3(kScanThreads), lds, st, pa);
    HIP_TRY(hipGetLastError());
    return HR_OK;
}

}  // namespace

int launch_persist(int mt, int dtype, int P, int cus, const PersistLaunch& pa, int lds, hipStream_t st) {
    if (mt == BF16 && dtype == BF16 && P == 16) return launch_t<BF16, BF16, 16>(cus, pa, lds, st);
    if (mt == F16 && dtype == F16 && P == 16) return launch_t<F16, F16, 16>(cus, pa, lds, st);
    if (mt == F16 && dtype == F32 && P == 4) return launch_t<F16, F32, 4>(cus, pa, lds, st);
    if (mt == BF16 && dtype == F32 && P == 4) return launch_t<BF16, F32, 4>(cus, pa, lds, st);
    return set_err(HR_E_UNSUPPORTED, "no persistent FILTER for this plan");
}

int launch_persist_post(PersistCtl* c, uint32_t e, hipStream_t st) {
    hipLaunchKernelGGL(k_persist_post, dim3(1), dim3(64), 0, st, c, e);
    HIP_TRY(hipGetLastError());
    return HR_OK;
}

int launch_persist_close(PersistCtl* c, hipStream_t st) {
    hipLaunchKernelGGL(k_persist_close, dim3(1), dim3(64), 0, st, c);
    HIP_TRY(hipGetLastError());
    return HR_OK;
}

int launch_persist_wait(PersistCtl* c, uint32_t e, uint32_t nwg, uint32_t* host_err, hipStream_t st) {
    hipLaunchKernelGGL(k_persist_wait, dim3(1), dim3(64), 0, st, c, e, nwg, host_err);
    HIP_TRY(hipGetLastError());
    return HR_OK;
}

}  // namespace hr
