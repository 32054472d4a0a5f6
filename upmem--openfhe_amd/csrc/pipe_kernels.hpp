// pipe_kernels.hpp -- the metric pipeline c = INTT(NTT(a) (.) b) at N = 2^16
// (DCRTPoly SwitchFormat -> Times -> SwitchFormat, dcrtpoly-impl.h:2518-2524,
// dcrtpoly.h:185-200) as ONE persistent launch instead of three.
//
// Why: the three-launch pipeline (k_tcols fwd -> k_block fused -> k_tcols inv)
// runs at the 1400 W package power cap, and moving its 56 HBM bytes per
// coefficient is the largest share of that power ("The clock
// is set by the package power cap").  32 of the 56 bytes are the two
// intermediates.  Here each XCD drains its own queue of work items in a
// software-pipelined order, so a polynomial tower's three passes run on the
// same XCD a few steps apart and its intermediates are re-read from that XCD's
// L2 / the Infinity Cache instead of HBM, and the HBM-bound column passes
// overlap the VALU-bound block passes.
//
// Work items.  A unit is one polynomial tower u = t * batch + b (512 KiB).
// Each unit has three phases of 16 items: F (k_tcols forward, one 16-column
// tile each), B (k_block fused, one 4096-element block each) and I (k_tcols
// inverse).  Queue x (XCD x) owns units u = x, x + 8, ... (the k-th: U_k) and
// hands out items in steps of 48: step s = { F(U_s), B(U_(s-L)), I(U_(s-2L)) }
// with lag L, so a B item is handed out 48 L items after the F items it
// depends on.  B(U) waits until all 16 F(U) items are done, I(U) until all
// 16 B(U) items are; dependencies only point to items handed out earlier, so
// every wait ends (an item is handed out only to a running workgroup, which
// finishes it) whatever the grid size and residency.
//
// Memory ordering (producer and consumer always on the same XCD, sharing its
// L2): a producer waits for its stores (s_waitcnt vmcnt(0)), then bumps the
// unit's counter with a relaxed L2 atomic; a consumer polls the counter with
// L1-bypassing loads, then runs an agent-scope acquire (buffer_inv sc1), so
// no load of the item can hit a stale L1 line.  The release side skips the L2
// write-back an agent-scope release would add (buffer_wbl2): no other XCD
// reads the data before the kernel ends.  The plan checks once that the
// queues map one-to-one onto XCDs (pipe_probe in ofhe_hip.hip) before it ever
// selects this kernel.
#pragma once
#include "ntt_kernels.hpp"

namespace ofhe {

// XCD (XCC) the calling wave runs on
__device__ __forceinline__ u32 xcc_id() {
    u32 x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    return x & 15;
}

constexpr u32 PIPE_PIECES = 16;  // items per phase of a unit (16-column tiles, 4096-element blocks)
constexpr u32 PIPE_STEP = 3 * PIPE_PIECES;
constexpr u32 PIPE_QSTRIDE = 32;  // u32 words between queue heads (one 128-byte line each)

struct PipeCtl {
    u32* head;    // [nq * PIPE_QSTRIDE] queue heads
    u32* done_f;  // [units] forward column tiles finished
    u32* done_b;  // [units] block-pass blocks finished
    u32* exited;  // [1] workgroups that have left the item loop
    u32* members; // [nq * PIPE_QSTRIDE] static mode: workgroups that joined each queue
    u32* err;     // [1] per plan: waits that gave up + queues left undrained (never expected)
    u32 units;    // batch * towers
    u32 lag;      // steps between a unit's phases (>= 1)
    u32 nq;       // queues = XCDs
    u32 pieces;   // pieces (tiles / blocks) per work item: 1, 2, 4, 8 or 16
    u32 wpq;      // 0: dynamic queue; else static, workgroups per queue
};

// workgroup-wide: wait until *ctr >= need, then (ACQ) acquire: the agent-scope
// fence invalidates this CU's L1 asynchronously, and the s_waitcnt after it
// holds the barrier until it has completed (MI355X_MICROARCH.md, "Consumer,
// always"); without ACQ every load of the handed-off data must bypass L1 (sc1)
template <bool ACQ>
__device__ __forceinline__ void pipe_wait(u32* ctr, u32 need, u32* err) {
    if (threadIdx.x == 0) {
        u32 spins = 0;
        while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < need) {
            __builtin_amdgcn_s_sleep(2);
            // ~1 s: a broken invariant, never a normal wait.  Once any wait has
            // given up, every later one returns at once, so the launch still
            // drains in about that second (wrong c, counted in err).
            if (++spins > (1u << 23) ||
                ((spins & 255) == 0 && __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
                __hip_atomic_fetch_add(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
        }
        if (ACQ) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
    }
    __syncthreads();
}

// workgroup-wide: every thread's stores have reached L2, then count the item's
// pieces
__device__ __forceinline__ void pipe_signal(u32* ctr, u32 pieces) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_fetch_add(ctr, pieces, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

#ifndef OFHE_PIPE_EARLY_CLAIM
#define OFHE_PIPE_EARLY_CLAIM 0
#endif
__device__ __forceinline__ void pipe_claim(u32* head, u32& nxt) {
    if (!OFHE_PIPE_EARLY_CLAIM && threadIdx.x == 0)
        nxt = __hip_atomic_fetch_add(head, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// HM, the hand-off mode of the intermediates: 0 acquire + plain loads, plain
// stores; 1 sc1 loads (no acquire), plain stores; 2 sc1 loads, non-temporal
// stores; 3 acquire + non-temporal loads and stores
template <bool SPQ, int HM>
__global__ __launch_bounds__(256, OFHE_KB_WAVES) void k_pipe(PlanArgs P, const u64* a, u64* c,
                                                             const u64* __restrict__ b, u32 batch, PipeCtl C) {
    OFHE_VGPR_FLOOR();
    __shared__ u64 lds[LDS_WORDS > TCOLS_LDS_WORDS ? LDS_WORDS : TCOLS_LDS_WORDS];
    __shared__ u32 s_next;
    const u32 tid = threadIdx.x;
    const u32 q = xcc_id() % C.nq;
    const u32 nu = C.units > q ? (C.units - q + C.nq - 1) / C.nq : 0;  // units of this queue
    const u32 ipp = PIPE_PIECES / C.pieces;  // items per phase of a unit
    const u32 total = nu ? (nu + 2 * C.lag) * 3 * ipp : 0;
    u32* head = C.head + PIPE_QSTRIDE * q;
    const SwSrc none{nullptr, 0, 0, nullptr, 1, 0};
    constexpr bool SC1 = HM == 1 || HM == 2;
    constexpr int OUT = (HM >= 2) ? 0 : 2;                  // IM bit 1: cached intermediate stores
    constexpr int IN = SC1 ? 4 : (HM == 3 ? 0 : 1);         // IM bits 0 / 2: plain or sc1 intermediate loads
    // dynamic (C.wpq = 0): items from the queue head, handed only to running
    // workgroups, so every wait ends whatever the residency.  Static
    // (OFHE_PIPE_STATIC, an A/B knob): the r-th workgroup of this XCD takes
    // items r, r + wpq, r + 2 wpq, ... with no claim per item; the lowest
    // unfinished item never waits, so it completes as long as all wpq
    // workgroups of the queue are resident (the grid is sized to that); a
    // concurrent kernel holding CU slots can stall it until the bounded wait
    // gives up, which err counts
    if (tid == 0) s_next = __hip_atomic_fetch_add(C.wpq ? C.members + PIPE_QSTRIDE * q : head, 1u, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    u32 item = __builtin_amdgcn_readfirstlane(s_next);  // wave-uniform: kept in SGPRs
    if (C.wpq && item >= C.wpq) item = total;             // more workgroups on this XCD than planned
    while (item < total) {
        // the next item is claimed when this one's loads are all consumed (its
        // last stores are in flight): a returning atomic issued earlier would
        // hold every load wait of the claiming wave behind its round trip
        // (vmcnt counts in order), OFHE_PIPE_EARLY_CLAIM = 1 claims at the top
        u32 nxt = 0;
#if OFHE_PIPE_EARLY_CLAIM
        if (!C.wpq && tid == 0) nxt = __hip_atomic_fetch_add(head, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#endif
        const u32 step = item / (3 * ipp), slot = item % (3 * ipp);
        const u32 ph = slot / ipp, grp = slot % ipp;
        if (step >= ph * C.lag && step - ph * C.lag < nu) {
            // every index below is wave-uniform; readfirstlane tells LLVM so,
            // which keeps the tower constants and table bases in scalar loads
            const u32 u = __builtin_amdgcn_readfirstlane(q + C.nq * (step - ph * C.lag));
            if (ph == 1) pipe_wait<!SC1>(C.done_f + u, PIPE_PIECES, C.err);
            if (ph == 2) pipe_wait<!SC1>(C.done_b + u, PIPE_PIECES, C.err);
            for (u32 k = 0; k < C.pieces; k++) {
                const u32 wid = __builtin_amdgcn_readfirstlane(u * PIPE_PIECES + grp * C.pieces + k);
                // a fresh copy of the thread index per piece: without it LLVM
                // hoists every phase's thread-index arithmetic (LDS and global
                // offsets) out of the loop, all of it stays live across all
                // three phases, and the kernel spills (312 B of scratch at 128
                // VGPRs; 116 VGPRs and no scratch with this)
                u32 ti = tid;
                asm volatile("" : "+v"(ti));
                if (k) __syncthreads();  // the previous piece's LDS reads are done
                if (ph == 0)
                    tcols_body<false, SPQ, false, 16, OUT>(P, a, c, batch, wid, none, lds, ti);
                else if (ph == 1)
                    block_body<MODE_FUSED, SPQ, 2, 0, IN | OUT>(P, c, c, b, batch, wid, lds, ti);
                else
                    tcols_body<true, SPQ, false, 16, IN>(P, c, c, batch, wid, none, lds, ti);
            }
            if (!C.wpq) pipe_claim(head, nxt);
            if (ph == 0) pipe_signal(C.done_f + u, C.pieces);
            if (ph == 1) pipe_signal(C.done_b + u, C.pieces);
        } else if (!C.wpq) {
            pipe_claim(head, nxt);
        }
        if (C.wpq) {
            item = __builtin_amdgcn_readfirstlane(item + C.wpq);  // uniform (nxt may hold a lane-0 claim)
            __syncthreads();  // LDS free
        } else {
            __syncthreads();  // LDS and s_next free
            if (tid == 0) s_next = nxt;
            __syncthreads();
            item = __builtin_amdgcn_readfirstlane(s_next);
        }
    }
    // audit by the last workgroup out: every queue with units was drained
    // (dynamic) or had all its planned workgroups (static); a queue no
    // workgroup ran on would leave its towers unwritten
    if (tid == 0 && __hip_atomic_fetch_add(C.exited, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1) {
        for (u32 x = 0; x < C.nq; x++) {
            const u32 n = C.units > x ? (C.units - x + C.nq - 1) / C.nq : 0;
            const bool bad =
                C.wpq ? __hip_atomic_load(C.members + PIPE_QSTRIDE * x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < C.wpq
                      : __hip_atomic_load(C.head + PIPE_QSTRIDE * x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <
                            (n + 2 * C.lag) * 3 * ipp;
            if (n && bad) __hip_atomic_fetch_add(C.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// one-time placement probe: the XCD of every workgroup of a k_pipe-sized grid
__global__ void k_pipe_probe(u32* xcc) {
    OFHE_VGPR_FLOOR();
    if (threadIdx.x == 0) xcc[blockIdx.x] = xcc_id();
}

}  // namespace ofhe
