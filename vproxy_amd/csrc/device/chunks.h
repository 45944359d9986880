// chunks.h -- the 64-item chunks a wave of a string or frame kernel works
// on: from a per-launch work-ticket counter (launch.h TicketRing), or the
// static grid-stride sequence without one.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dev_common.h"
#include "launch.h"

namespace vcd {

// The 64-item chunks of a launch, in wave-uniform order: taken a ticket at
// a time from the launch's ticket counter (launch.h TicketRing) or, without
// one, the static grid-stride sequence.  A ticket is a run of chunks: the
// first tickets cover kPerTicket chunks (1024 items), which keeps the
// counter's same-address atomics (served one at a time at the memory side)
// far below the kernel's rate -- one ticket per 64-name chunk made the hint
// pass 3.6x slower, four per ticket 17 % slower, 64 per ticket 39 % slower
// (too few tickets per wave); the last chunks, kTailRounds small tickets per
// wave, go kTailChunks at a time, so the launch does not end one whole big
// ticket after most waves ran out of work (a C4 pool pass is only ~2.3 big
// tickets per wave).  Tails of 4-chunk tickets, two per wave: C4 0.813 ->
// 0.803 ms, DNS 1.10 -> 1.06, the C5 step 6.13 -> 6.03-6.06 ms; 1- and
// 2-chunk tails lose to their extra atomics, 8-chunk ones end too coarsely
// (profiles/r03_ab_ticket.txt).  Round 4, once the hint / DNS kernels had no
// call in their loops and a chunk cost less: 24-chunk big tickets and one
// round of 8-chunk tail tickets -- C4 0.762 -> 0.705 ms, SNI 0.635 -> 0.580,
// mirror 2.495 -> 2.397, DNS 0.892 -> 0.880 (profiles/r04_ab_ticket_sweep*.txt;
// 32-chunk tickets lose on every kernel).  With little work per chunk the
// single counter itself is the cost: the C4 pass without its scan ran 0.474
// ms on tickets against 0.317 ms on the static split (r04_ab_hint_ablation.txt),
// and eight counters on separate lines lost to the one counter once the scan
// was back (r04_ab_part_tickets.txt).
// Every wave takes exactly one out-of-range ticket (its last), so the wave
// holding ticket ntickets + nwaves - 1 is the last taker of the launch and
// resets the counter for the slot's next launch.
// VC_DNSD_TICKETS: dnsd_kernel takes its chunks from the work tickets
#ifndef VC_DNSD_TICKETS
#define VC_DNSD_TICKETS 1
#endif
#ifndef VC_TICKET_CHUNKS
#define VC_TICKET_CHUNKS 24
#endif
#ifndef VC_TICKET_TAIL
#define VC_TICKET_TAIL 8
#endif
constexpr int64_t kPerTicket = VC_TICKET_CHUNKS;
constexpr int64_t kTailChunks = VC_TICKET_TAIL;     // 0: big tickets to the end
#ifndef VC_TICKET_TAIL_ROUNDS
#define VC_TICKET_TAIL_ROUNDS 1
#endif
constexpr int64_t kTailRounds = VC_TICKET_TAIL_ROUNDS;

// Ticket t -> its chunk run: big tickets [B t, B t + B) up to chunk head,
// then tail tickets of kTailChunks.  `end` is the end of the wave's current
// run (wave-uniform).
// S (percent): that share of the chunks goes to the waves first, in
// contiguous blocks of equal size without a ticket; the rest by tickets.  A
// wave's static block is read as one stretch of the blob, and the ticket
// counter sees fewer takes: C4 0.699 -> 0.626 ms at 60 %, DNS 0.879 -> 0.809
// at 50 %, SNI 0.579 -> 0.548 and mirror 2.39 -> 2.27 ms at 25 %, the DNS
// drain loop 4.00 -> 3.93 ms at 60 %, the C5 step 6.02 -> 5.95 ms
// (profiles/r04_ab_ticket_static*.txt); each kernel takes its best share.
template <int64_t P = kPerTicket, int64_t T = kTailChunks, int64_t R = kTailRounds, int S = 0>
struct ChunksT {
    uint32_t* ticket;
    int64_t nchunks;
    int64_t head = 0;              // chunks covered by big tickets
    int64_t nbig = 0;              // big tickets
    int64_t ntickets = 0;
    int64_t end = 0;
    int64_t s0 = 0;                // chunks [0, s0) are the waves' static blocks
    int64_t sb = 0;                // static block per wave
    __device__ ChunksT(uint32_t* t, int64_t nc) : ticket(t), nchunks(nc) {
        const int64_t nwaves = int64_t(gridDim.x) * (blockDim.x / 64);
        if (S > 0 && t) {
            sb = nc * S / 100 / nwaves;
            s0 = sb * nwaves;
        }
        const int64_t rest = nc - s0;
        const int64_t tail = T ? nwaves * T * R : 0;
        head = rest > tail ? (rest - tail) / P * P : 0;
        if (!T) head = rest;
        nbig = (head + P - 1) / P;
        ntickets = nbig + (T ? (rest - head + T - 1) / T : 0);
        head += s0;
    }
    __device__ int64_t take() {
        uint32_t t = 0;
        if ((threadIdx.x & 63) == 0) {
            t = atomicAdd(ticket, 1u);
            const uint32_t nwaves = gridDim.x * (blockDim.x / 64);
            // a slot left nonzero by an aborted launch (launch.h TicketRing)
            VC_CHECK(t <= uint32_t(ntickets) + nwaves - 1, 304, t, uint32_t(ntickets) + nwaves);
            if (t == uint32_t(ntickets) + nwaves - 1) atomicExch(ticket, 0u);
        }
        const int64_t tk = int64_t(__shfl(t, 0, 64));
        int64_t start;
        if (tk < nbig) {
            start = s0 + tk * P;
            end = start + P < head ? start + P : head;
        } else {
            start = head + (tk - nbig) * (T ? T : 1);
            end = start + T;
        }
        if (end > nchunks) end = nchunks;
        return start < nchunks ? start : nchunks;
    }
    __device__ int64_t first(int w) {
        const int64_t gw = int64_t(blockIdx.x) * (blockDim.x / 64) + w;
        if (ticket && sb > 0) {
            end = (gw + 1) * sb;
            return gw * sb;
        }
        return ticket ? take() : gw;
    }
    __device__ int64_t next(int64_t c) {
        if (!ticket) return c + int64_t(gridDim.x) * (blockDim.x / 64);
        return c + 1 < end ? c + 1 : take();
    }
    // c + 1 is this wave's next chunk (same ticket)
    __device__ bool paired(int64_t c) const { return ticket && c + 1 < end; }
};

// the string and frame kernels' layout (the constants above)
using Chunks = ChunksT<>;

}  // namespace vcd

namespace vc {
// The work-ticket slot of one launch (null without a ring).
inline uint32_t* launch_ticket(const LaunchCfg& c) {
    return c.tickets ? c.tickets->next(c.stream) : nullptr;
}
}  // namespace vc
