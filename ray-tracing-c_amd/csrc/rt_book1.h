// rt_book1.h — the fast path for sphere/BVH scenes (reference scenes 0 and 1: the headline
// Book-1 final scene).  Same arithmetic as rt_device.h (bit-exact with the reference); different
// execution structure, designed for a 64-wide CDNA4 wavefront:
//
//  * persistent lanes + wave-level work stealing: a lane that finishes its work item takes the next
//    one (one atomic per wave per refill: ballot + mbcnt), longest items first;
//  * one flattened loop per lane over (sample, bounce): per wave iteration either a few traversal
//    steps for the lanes still tracing, or one shading pass once enough lanes wait for it;
//  * the world in traversal preorder (stackless scan with skips), staged once per workgroup in LDS;
//  * the path record is a list of material ids (albedo of a Solid texture is a function of the
//    material) in registers (two 4-id chunks) + a per-lane global spill area for deep paths; the
//    colour is folded innermost-first at path end exactly like the recursion;
//  * the heaviest chain items run on whole waves (coop_items) in the chain kernel's first waves;
//  * chain render (kMode 2): a pixel's sample stream can be cut into segments that run as separate
//    work items and meet again exactly (ChainPx below) -- the frame is no longer bound by the
//    longest pixel's sequential chain when it is split over many GPUs.
//
// Eligibility (host-checked, rt_kernel.hip: book1_eligible): spheres only, BVH nodes, lists only at
// the root, Lambertian/Metal/Dielectric with Solid albedo, no lights/emission/textures/transforms.
#pragma once
#include "rt_device.h"

namespace rt {
namespace b1 {

constexpr int kBlock = 256;
constexpr int kWaves = kBlock / 64;

struct FastMat {   // 32 B: material resolved to what the Book-1 path needs
  float albedo[3];  // Solid texture colour; (1,1,1) for Dielectric
  float param;      // fuzz / eta
  int32_t tag;
  int32_t pad[3];
};

// ================================================================ chain render (kMode 2)
// A pixel's samples share one pcg32 stream (src/raytracing.c:93-124): sample s starts at stream
// offset o_s and draws D(o_s), so o_{s+1} = o_s + D(o_s), and a sample's colour and draw count are
// functions of its start offset alone.  A split pixel's stream is cut into K segments; segment k
// is one work item (a chain) that starts at offset B_k = k * seg_len and computes sample after
// sample from there.  Segment 0 starts on the true chain (offset 0).  Any other chain starts
// mid-sample (garbage) but, sampling the same D, lands on an offset of the true chain within a few
// samples (the Kruskal count: scripts/couple_sim.c measured 1-15 samples per cut on the headline
// frame, against a segment length of 60-500).  So:
//  * segment k >= 1 stores each sample as a record (colour, end offset) in its own list;
//  * chain k, once past B_{k+1}, compares each of its sample start offsets with the start offsets
//    of its successor's records (start of record c = end of record c-1, B for c = 0); at the first
//    equal offset x the two chains coincide from x on: chain k ends there with a link (t, c) to the
//    successor's record c ("coupled"; a successor that ended itself passes its own link on);
//  * a chain ends at its record capacity (its list is full), and the last chains end once the link
//    structure shows that the pixel's spp true samples exist (chain_walk);
//  * chain_fold_kernel (after the launch) follows the links from segment 0 -- whose chain adds its
//    own samples in registers -- summing the records in sample order, the reference's summation
//    order, so the pixel is bit-identical; a pixel whose links end early (a list that filled up,
//    a misestimated stream) is finished by a continuation item that runs the true chain on from
//    the exact position the fold reached.
// Records are exchanged between chains running concurrently on different XCDs: the end offsets
// (the only words read during the launch) are written and read with relaxed agent-scope atomics
// (no cache maintenance; a reader that sees the fill value or a running segment just retries at
// its next sample boundary); colours are plain stores read by the fold after the launch.
struct ChainPx {       // 32 B per pixel of a chain launch (chain_plan_kernel)
  uint32_t K;          // segments (K == 1: unsplit, not read by the chains)
  uint32_t seg_len;    // segment k starts at stream offset k * seg_len (even)
  uint32_t rec0;       // segment k >= 1 keeps its records at [rec0 + (k - 1) * cap, + seg_cap)
  uint32_t cap;        // records per segment
  uint32_t end0;       // segment k's end word at ch_seg[end0 + k]
  uint32_t check;      // a segment >= 1 looks for the pixel's end once it holds this many records
  uint32_t cap_last;   // records of the last segment (it takes whatever remains of the stream)
  uint32_t pad;
};
constexpr uint32_t kNone = 0xffu;  // no successor
struct ChainCont {     // 32 B: a continuation item -- the true chain from an exact position
  uint32_t pix, o, s, pad;
  float acc[4];
};
// Migration (tail of a launch): a lane whose wave has run out of work items and has few live lanes
// left hands its item over at a sample boundary -- the whole state there is (pcg32 state and offset,
// samples / records so far, colour sum, coupling cursor) -- to a wave whose lanes have all finished,
// which runs it on to the end with whole-wave traces (render_item_coop).
// Control words at V.mig (uint32): [0] done: the launch's finished items; [1] helpers: waves that
// have become helpers; [2] fault injection (tests): items dropped so far; then kMigBoxes mailboxes of
// one 128-B line each:
//   push / pop: indices into the mailbox's part of the queue; credits: its idle helpers not yet
//   claimed by a push (a lane pushes only against a credit, so a queued item always has a helper;
//   a helper leaves only by taking back a credit nobody has claimed);
//   finished: set once every item is done (the helpers' exit).
// Helpers poll only their own mailbox's line, rarely: thousands of idle waves polling one address
// would swamp that memory channel and slow every working lane (measured: +30 % at N = 8).
// After the launch, chain_check_kernel compares [0] with the launch's item count: a launch that
// finished fewer items than it was given is reported through the scene's status word.
constexpr int kMigBoxes = 64, kMigBoxWords = 32;
enum : int {
  kMigDone = 0, kMigHelpers = 1, kMigDropped = 2, kMigBox0 = 64,
  kMigStat = 4,  // (diagnostic build, RT_DEBUG: 6 u64 of migrated items' rays and clocks, words 4-15)
  kMigPush = 0, kMigPop = 1, kMigCredits = 2, kMigFinished = 3
};
constexpr int kMigWords = kMigBox0 + kMigBoxes * kMigBoxWords;
constexpr int kMigMode = 2;  // the launches that migrate: chain launches (kMode 2)
struct MigRec {       // 64 B
  uint64_t state;     // pcg32 state at the sample boundary (inc follows from the pixel's seed)
  uint32_t n;         // stream offset
  uint32_t pix, seg, s, tc, st;
  float acc[3];
  uint32_t ready;     // the launch's epoch, written last (release); the helper's acquire load waits for it
  uint32_t pad[2];
};
constexpr uint32_t kItemUnsplit = 0x80000000u;  // ch_items[].y: K == 1, the whole pixel
constexpr uint64_t kEndEnded = 1ull << 63;      // end word: the segment's chain has ended
constexpr uint64_t kEndNoLink = 1ull << 62;     //   ... without coupling (pixel complete / list full)
constexpr uint32_t kRecFill = 0xffffffffu;      // a record's end word (ch_col .w) before the record is written
constexpr uint32_t kNoTarget = 0xff000000u;     // coupling cursor (t << 24 | c): none
constexpr int kMaxSeg = 255;                    // t fits 8 bits (host: chain planner caps K lower)
RT_D uint32_t end_n(uint64_t w) { return (uint32_t)(w >> 32) & 0x3fffffffu; }
RT_D uint32_t end_t(uint64_t w) { return (uint32_t)w >> 24; }
RT_D uint32_t end_c(uint64_t w) { return (uint32_t)w & 0xffffffu; }
RT_D uint64_t end_word(uint32_t n, bool link, uint32_t tc) {
  return kEndEnded | (link ? 0ull : kEndNoLink) | ((uint64_t)(n & 0x3fffffffu) << 32) | (link ? tc : 0u);
}
RT_D float u2f(uint32_t u) { return __builtin_bit_cast(float, u); }  // (host and device)
RT_D uint32_t f2u(float f) { return __builtin_bit_cast(uint32_t, f); }
RT_D uint32_t ld_rel(const uint32_t *p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
RT_D uint64_t ld_rel64(const uint64_t *p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
RT_D void st_rel(uint32_t *p, uint32_t v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
RT_D void st_rel64(uint64_t *p, uint64_t v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
// One 16-B write-through (sc1) store, the 16-B form of st_rel: the other XCDs' relaxed agent loads
// (global_load sc1) of any of its words see the stored value (MI355X_MICROARCH.md, visibility: 16-B
// sc1 stores observed untorn; one fabric write, where a 4-B sc1 store costs ~6x per byte).  The asm
// ends with s_nop 1 so the next instruction cannot overwrite the data registers before the store reads
// them.
RT_D void st_rel128(float4 *p, float4 v) {
#if defined(__HIP_DEVICE_COMPILE__)
  typedef float f4v __attribute__((ext_vector_type(4)));
  const f4v x = {v.x, v.y, v.z, v.w};
  asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(x) : "memory");
#else
  // (the host harnesses: tests/native/chain_sim.cpp runs the protocol single-threaded)
  *p = v;
#endif
}
RT_D uint32_t ld_acq(const uint32_t *p) { return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT); }

struct Book1View {
  DScene S;                  // full scene (global memory): sphere aux data, camera
  const FastMat *mats;
  const float4 *items9_g;    // the world in traversal preorder, 2 float4 per item (trav_step_v9)
  int32_t n_items9, n_items9_alloc;  // items, and items incl. the zero pad item at the end
  int32_t row0, row_stride, n_rows;
  int32_t *work_counter;     // zeroed before each launch
  int32_t shade_batch;       // shade once this many lanes of a wave are waiting
  uint32_t *cost_out;        // cost pre-pass: traversal steps per work item, or null
  uint32_t cost_budget;      // cost pre-pass: steps after which a pixel's estimate is extrapolated
  uint32_t *draw_out;        // cost pre-pass (kMode 1): pcg32 draws per work item
  // the cost pre-pass's samples are the pixel's first samples: it leaves each pixel's colour sum and
  // position there (pre_word: stream offset | samples << 24), and the chain launch's segment 0 / unsplit
  // items go on from it instead of rendering them again (null: off)
  float4 *pre_state;
  // the cost pre-pass of a chain launch: its waves, once out of pixels, set the record arena's first
  // *clean_n records (what the previous chain launch reserved) back to kRecFill (null: off)
  float4 *clean_col;
  const uint32_t *clean_n;
  const uint32_t *n_coop;    // chain launches: the first *n_coop of ch_items go to whole waves
  int32_t *coop_counter;     //   (coop_items), claimed through this counter
  const uint32_t *coop_waves_dev;  // by the first *coop_waves_dev waves of the grid
  uint64_t *spill;           // [chunk][global lane]: a deep path's older 4-id chunks (Record)
  int32_t spill_lanes;
  int32_t n_bf_leaves;       // whole-wave pixels: leaves for bf_candidate; 0: off (coop_trace9 instead)
  const struct BfCut *bf_cuts;  // and its subtree cuts (bf_candidate_cut); n_bf_cuts 0: every leaf each ray
  int32_t n_bf_cuts;
  uint32_t *px_time;         // diagnostic (RT_PX_TIME=1): per work item {start, end, migrated}, wall_clock64 low bits
  // chain render (kMode 2)
  const ChainPx *ch_px;      // per pixel
  const uint2 *ch_items;     // {pixel, segment | kItemUnsplit}: whole-wave items first, then lanes'
  const uint32_t *ch_n_items;
  uint64_t *ch_seg;          // segment end words (0: running)
  float4 *ch_col;            // records: colour, end offset (bits; kRecFill until written)
  float4 *ch_acc0;           // per pixel: segment 0's colour sum when it coupled
  uint32_t *seg_time;        // diagnostic (RT_PX_TIME=1): per segment {start, end, migrated} at end0 + k
  const ChainCont *ch_cont;  // continuation launch: items from here (else null)
  const uint32_t *ch_n_cont;
  // migration (MigRec): control words, queue, its capacity; mig_live: a wave with at most this many
  // live lanes (and no work items left) migrates them; 0: off
  uint32_t *mig;
  MigRec *mig_q;
  uint32_t mig_cap;
  int32_t mig_live;
  uint32_t mig_epoch;  // per launch (> 0): marks the queue entries this launch wrote
  int32_t mig_idle;    // migrate only once more waves than this have become helpers
  uint32_t walk_mask;  // a segment past its check looks for its pixel's end every walk_mask + 1 samples
  uint32_t mig_poll;   // a sparse wave reads the helper count every this many ticks until the gate opens
  int32_t mig_sleep;     // helpers poll their mailbox every mig_sleep * ~3.4 us
  unsigned long long *loop_stats;  // diagnostic builds (-DRT_LOOP_STATS): per-launch loop counters
  int32_t mig_max_help;  // at most this many finished waves stay as helpers; the others leave.  Resident
                         // idle waves slow the working ones (measured: all 5120 waves of a grid kept
                         // resident made N = 8 shares 20 % slower, however rarely they polled)
  uint32_t mig_drop;     // fault injection (tests only): helpers drop this many popped items unrun
  uint64_t mig_wait;     // a helper idle this long (wall_clock64 ticks, 100 MHz) offers to leave
};
// a record's end word (ch_col[i].w), read as st_rel128 published it
RT_D uint32_t rec_end(const Book1View &V, uint32_t i) { return ld_rel((const uint32_t *)&V.ch_col[i] + 3); }

using rt::pre_word;
// A chain launch's item that starts the pixel's true chain at offset 0 -- segment 0 of a split pixel, or
// an unsplit pixel -- goes on from the pre-pass's position instead: same samples, same summation order
// (acc = ((0 + c_0) + c_1) + ...), so the pixel is bit-identical and its first samples are not rendered
// twice.
RT_D void pre_resume(const Book1View &V, int64_t pix, uint32_t seg, Pcg32 &g, uint32_t &s, f3 &acc) {
  if (!V.pre_state || !((seg & kItemUnsplit) || seg == 0u)) return;
  const float4 p = V.pre_state[pix];
  const uint32_t w = __builtin_bit_cast(uint32_t, p.w), n = w >> 24;
  if (n == 0u) return;
  g.skip(w & 0xffffffu);
  s = n;
  acc = mk(p.x, p.y, p.z);
}

// ---------------------------------------------------------------- chain segments
RT_D uint32_t seg_start(const ChainPx &P, uint32_t t) { return t * P.seg_len; }
RT_D uint32_t seg_cap(const ChainPx &P, uint32_t k) { return k + 1u < P.K ? P.cap : P.cap_last; }
RT_D uint32_t rec_index(const ChainPx &P, uint32_t t, uint32_t c) { return P.rec0 + (t - 1u) * P.cap + c; }
RT_D uint32_t seg_next(const ChainPx &P, uint32_t t) { return t + 1u < P.K ? t + 1u : kNone; }  // or kNone

// ---------------------------------------------------------------- pixel output
// quantize one pixel (src/raytracing.c:127-131): mean, gamma 2, clamp-macro semantics, truncate
RT_D uint8_t quantize(float sum, float spp_f) {
  float v = sqrtf(sum / spp_f);
  v = v > 0.0f ? v : 0.0f;
  v = v < 0.999f ? v : 0.999f;
  return (uint8_t)(int)(256.0f * v);
}
RT_D void write_pixel(uint8_t *dst, f3 acc, int spp) {
  const float spp_f = (float)spp;
  dst[0] = quantize(acc.x, spp_f);
  dst[1] = quantize(acc.y, spp_f);
  dst[2] = quantize(acc.z, spp_f);
}

// ---------------------------------------------------------------- per-lane ray state
typedef float f2v __attribute__((ext_vector_type(2)));

struct Lane {         // plain scalars: an f3 member here was kept in scratch by the compiler
  float ox, oy, oz;   // current ray origin
  float dx, dy, dz;   // direction
  float ix, iy, iz;   // 1/d (hoisted: same IEEE division as AABB_hit)
  float a, tmax;      // |d|^2, closest hit so far
  float ra;           // refined reciprocal of a (div_core), hoisted per ray
  bool fast;          // a in the range where div_core == '/'
  int32_t hit;        // the hit leaf item's byte offset (as cur), or -1
  uint32_t cur;       // preorder item being visited (byte offset: index x 16)
};

// AABB_hit with the slabs evaluated together: t_min / t_max only tighten and fmaxf/fminf ignore a
// NaN operand, so testing tmax <= tmin once after all three slabs returns exactly what the
// reference's per-slab early exit returns.  (lo,hi) pairs are packed: one v_pk_add + v_pk_mul per
// axis.  Swap on a negative 1/d as the reference does (select, not min/max, for NaN parity).
RT_D bool aabb_packed(float4 a, float4 b, const Lane &L, float tmin) {
  const f2v px = (f2v){(a.x - L.ox) * L.ix, (a.y - L.ox) * L.ix};
  const f2v py = (f2v){(a.z - L.oy) * L.iy, (a.w - L.oy) * L.iy};
  const f2v pz = (f2v){(b.x - L.oz) * L.iz, (b.y - L.oz) * L.iz};
  const float t0x = L.ix < 0 ? px.y : px.x, t1x = L.ix < 0 ? px.x : px.y;
  const float t0y = L.iy < 0 ? py.y : py.x, t1y = L.iy < 0 ? py.x : py.y;
  const float t0z = L.iz < 0 ? pz.y : pz.x, t1z = L.iz < 0 ? pz.x : pz.y;
  const float lo = fmaxf(fmaxf(fmaxf(tmin, t0x), t0y), t0z);  // (never NaN: tmin is not)
  // hi = fminf(fminf(fminf(tmax, t1x), t1y), t1z) = fminf(tmax, m): "hi <= lo" iff "tmax <= lo" or
  // "m <= lo" (m NaN only when all three are, and then hi = tmax).  Testing the two separately spares
  // the canonicalisation of tmax (a loop-carried value) that fminf(tmax, ...) costs in every step.
  const float m = fminf(fminf(t1x, t1y), t1z);
  return !(L.tmax <= lo) & !(m <= lo);
}

// Sphere_hit (src/hittable.c:120-151) as the reference writes it: the diagnostics' yardstick for
// the exact fast cores below (rt_diag_arith).
RT_D void sphere_test_lane(const float4 *sph, uint32_t ref, Lane &L, float tmin) {
  const int idx = (int)(ref & 0x7fff);
  const float4 s = sph[idx];
  const f3 oc = sub(mk(L.ox, L.oy, L.oz), mk(s.x, s.y, s.z));
  const float b = dot(oc, mk(L.dx, L.dy, L.dz));
  const float c = dot(oc, oc) - s.w;
  const float disc = b * b - L.a * c;
  if (disc < 0) return;
  const float sq = sqrtf(disc);
  float root = (-b - sq) / L.a;
  if (root <= tmin || root >= L.tmax) {
    root = (-b + sq) / L.a;
    if (root <= tmin || root >= L.tmax) return;
  }
  L.tmax = root;
  L.hit = idx;
}

// exact fast arithmetic: sqrt_core / recip_core / div_core and their ranges live in rt_device.h
using rt::div_core;
using rt::kDivHi;
using rt::kDivLo;
using rt::kNumHi;
using rt::kSqrtLo;
using rt::recip_core;
using rt::sqrt_core;

// Sphere_hit (src/hittable.c:125-150) with the exact cores; lanes outside their ranges (NaN,
// huge numerators, tiny discriminants, degenerate rays) evaluate the reference expression.
RT_D void sphere_test_data(float4 s, int idx, Lane &L, float tmin) {
  const f3 oc = sub(mk(L.ox, L.oy, L.oz), mk(s.x, s.y, s.z));
  const float b = dot(oc, mk(L.dx, L.dy, L.dz));
  const float c = dot(oc, oc) - s.w;
  const float disc = b * b - L.a * c;
  if (disc < 0) return;
  float sq = sqrt_core(disc);
  float r1 = div_core(-b - sq, L.a, L.ra), r2 = div_core(-b + sq, L.a, L.ra);
  // (bitwise, not short-circuit: one straight-line guard instead of nested branches)
  const bool ok = (int)L.fast & ((int)(disc == 0.0f) | ((int)(disc >= kSqrtLo) & (int)(disc <= __FLT_MAX__))) &
                  (int)(fabsf(-b - sq) <= kNumHi) & (int)(fabsf(-b + sq) <= kNumHi);
  if (__builtin_expect(!ok, 0)) {
    sq = sqrtf(disc);
    r1 = (-b - sq) / L.a;
    r2 = (-b + sq) / L.a;
  }
  // the reference tries root 1, then root 2, each rejected when (root <= t_min || root >= t_max)
  const bool take1 = !(r1 <= tmin || r1 >= L.tmax), take2 = !(r2 <= tmin || r2 >= L.tmax);
  if (take1 || take2) {
    L.tmax = take1 ? r1 : r2;
    L.hit = idx;
  }
}

// ---------------------------------------------------------------- stackless preorder traversal
// The reference's closest-hit recursion (HittableList_hit over the root items, BVHNode_hit = own box,
// then left, then right: src/hittable.c:74-88, :266-277) visits the hittables in the preorder of the
// world graph, skipping a node's whole subtree when its box misses.  The preorder is a flat item
// array, so the traversal is a scan with skips -- no stack, one item per step:
//   node item:  q0 = (lo.x, hi.x, lo.y, hi.y), q1 = (lo.z, hi.z, skip, 0)   next = hit ? p+1 : p+skip
//   leaf item:  q0 = (cx, cy, cz, r^2),        q1 = (-, -, -, idx | 1<<31)   Sphere_hit, next = p+1
// (skip = 1 + the node's subtree size in items).  The box test sees exactly the reference's t_max:
// every item before p in preorder that the reference would test has been tested, in order.
constexpr uint32_t kLeaf9 = 0x80000000u;
// Sibling leaves (RT_LEAF_PAIR): a leaf item whose successor in preorder is a leaf too (the two children
// of an n == 2 node, src/hittable.c:294-299) carries kLeafPair, and the step tests both spheres -- the
// second at the t_max the first left, as BVHNode_hit does (src/hittable.c:270-276) -- so a lane spends
// one step on the pair instead of two.  The leaf's sphere index sits in the bits below (kLeafIdx).
constexpr uint32_t kLeafPair = 0x40000000u, kLeafIdx = 0x3fffffffu;
#ifndef RT_LEAF_PAIR
#define RT_LEAF_PAIR 0
#endif
constexpr bool kPairLeaves = RT_LEAF_PAIR != 0;
// Items are stored as two arrays (q0 of every item, then q1 of every item: na = V.n_items9_alloc
// apart): a ds_read_b128 lane group (16 lanes, one 256-B bank row) then spreads random items over 16
// slots, where 32-B interleaved items use only 8 of them (more bank conflicts on the step's read).
RT_D float4 it_q0(const float4 *items, uint32_t p) { return items[p]; }
RT_D float4 it_q1(const float4 *items, int na, uint32_t p) { return items[(uint32_t)na + p]; }

// L.cur, na16 and n16 are byte offsets (item index x 16): na16 = 16 V.n_items9_alloc, n16 = 16 V.n_items9
// (hoisted by the caller, in VGPRs) -- the step then needs no index scaling.
// (Leaves waiting for company -- a lane at a leaf running its sphere test only once 8 / 16 / 32 lanes
// sit at leaves, the node lanes going on meanwhile -- measured 1 / 6 / 24 % slower, r04: the waiting
// lanes' latency costs more than the sphere block saves.)
RT_D bool trav_step_v9(const float4 *items, uint32_t na16, uint32_t n16, Lane &L, float tmin) {
  const uint32_t p = L.cur;
  typedef float f4v __attribute__((ext_vector_type(4)));
  const char *base = (const char *)items;
  f4v v0 = *(const f4v *)(base + p), v1 = *(const f4v *)(base + na16 + p);
  // both halves in one LDS round trip: without this the compiler sinks the q1.xy / q1.z reads into
  // the branches that use them, i.e. three dependent round trips per step.  (Reading the successor
  // one step ahead measured slower: its moves and the re-read after a skip cost more than the latency.)
  // (whole 128-bit tuples: per-component constraints made the compiler shuffle registers after the loads)
  asm volatile("" : "+v"(v0), "+v"(v1));
  const float4 q0 = make_float4(v0.x, v0.y, v0.z, v0.w), q1 = make_float4(v1.x, v1.y, v1.z, v1.w);
  const uint32_t w = __float_as_uint(q1.w);
  // (branches, not both tests straight-line for every lane: a wave's lanes are mostly at one kind --
  // the straight-line step measured 1.3x slower)
  uint32_t next = p + 16u;
  if (w & kLeaf9) {
    f4v u = {0.0f, 0.0f, 0.0f, 0.0f};
    if (kPairLeaves) u = *(const f4v *)(base + p + 16u);  // the successor's q0 (in bounds: the pad item)
    sphere_test_data(q0, (int)p, L, tmin);  // (the hit is the leaf's item: its q1 holds 1/r and the material)
    if (kPairLeaves && (w & kLeafPair)) {
      sphere_test_data(make_float4(u.x, u.y, u.z, u.w), (int)(p + 16u), L, tmin);
      next = p + 32u;
    }
  } else {
    if (!aabb_packed(q0, q1, L, tmin)) next = p + (__float_as_uint(q1.z) << 4);
  }
  L.cur = next;
  return next >= n16;
}

// ---------------------------------------------------------------- path record
// The path's material ids in push order, in chunks of 4 (16 bits each, newest in the low bits):
// r0 = the current chunk, r1 = the previous one; older chunks go to the per-lane spill area as one
// u64 each (one 8-byte store per 4 bounces beyond the 8th, instead of a 2-byte store per bounce).
// The spill area has max(0, ceil(max_depth / 4) - 2) chunks per lane (host: book1_upload).
struct Record {
  uint64_t r0, r1;
  int n;  // ids pushed
};

RT_D void rec_push(const Book1View &V, Record &R, uint32_t id, int glane) {
  if ((R.n & 3) == 0 && R.n > 0) {  // r0 is a complete chunk: start a new one
    if (R.n >= 8) V.spill[(int64_t)((R.n >> 2) - 2) * V.spill_lanes + glane] = R.r1;  // deep paths only
    R.r1 = R.r0;
    R.r0 = 0;
  }
  R.r0 = (R.r0 << 16) | id;
  R.n++;
}

// c = a_k * c for k = n-1 .. 0 (newest first), the recursion's evaluation order
RT_D f3 rec_fold_chunk(const Book1View &V, uint64_t w, int cnt, f3 c) {
  for (int k = 0; k < cnt; k++) {
    const FastMat &m = V.mats[(uint32_t)(w & 0xffff)];
    c = add(mk(0.0f, 0.0f, 0.0f), mul(ld3(m.albedo), c));
    w >>= 16;
  }
  return c;
}
RT_D f3 rec_fold(const Book1View &V, const Record &R, f3 c, int glane) {
  if (R.n == 0) return c;
  const int cnt0 = R.n - (((R.n - 1) >> 2) << 2);  // ids in the current chunk, 1..4
  c = rec_fold_chunk(V, R.r0, cnt0, c);
  if (R.n > cnt0) c = rec_fold_chunk(V, R.r1, 4, c);
  for (int q = ((R.n - 1) >> 2) - 2; q >= 0; q--)  // spilled chunks, newest first
    c = rec_fold_chunk(V, V.spill[(int64_t)q * V.spill_lanes + glane], 4, c);
  return c;
}

// ---------------------------------------------------------------- scattering (Book-1 materials)
RT_D f3 scatter(const FastMat &m, f3 normal, bool front, f3 r_in, Pcg32 &g) {
  if (m.tag == RT_MAT_LAMBERTIAN) {  // src/material.c:23-37
    const Onb b = onb_from_w(normal);
    const float r1 = g.f32();
    const float r2 = g.f32();
    const float phi = (2.0f * kPi) * r1;
    float sphi, cphi;
    rtm::sincosf(phi, &sphi, &cphi);
    const float sq = sqrtf(r2);
    return onb_local(b, mk(cphi * sq, sphi * sq, sqrtf(1.0f - r2)));
  }
  if (m.tag == RT_MAT_METAL) {  // src/material.c:48-58
    const f3 refl = reflect(normalize(r_in), normal);
    const f3 out = add(refl, scale(rand_unit_vector(g), m.param));
    return dot(out, normal) < 0.0f ? refl : out;
  }
  // DIELECTRIC, src/material.c:62-86
  float eta = m.param;
  if (front) eta = 1.0f / eta;
  const f3 v = normalize(r_in);
  const float cos_t = fminf(-dot(v, normal), 1.0f);
  const float sin_t = sqrtf(1.0f - cos_t * cos_t);
  float sch = (1.0f - eta) / (1.0f + eta);
  sch *= sch;
  sch += (1 - sch) * rtm::powf(1.0f - cos_t, 5.0f);
  if (eta * sin_t > 1.0f || sch > g.f32()) return reflect(v, normal);
  const f3 perp = scale(add(v, scale(normal, cos_t)), eta);
  const f3 para = scale(normal, -sqrtf(fabsf(1.0f - dot(perp, perp))));
  return add(perp, para);
}

// ---------------------------------------------------------------- whole-wave traces
// For the few work items whose sequential chain is far longer than the launch's fair share, a whole
// wave traces each ray: every box interval and every sphere root is independent of t_max, so the
// lanes compute them in parallel and wave-uniform logic recovers the reference's answer.
RT_D float lane_bcast(float x, int src) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), src)); }

struct CoopRay {  // wave-uniform copy of the traced ray
  float ox, oy, oz, dx, dy, dz, ix, iy, iz, a, ra;
  bool fast;
};

// Sphere_hit's accepted root for this sphere, independent of t_max: q1 unless q1 <= t_min, then q2
// (the two-root sequence of Sphere_hit, since q1 <= q2); "no root" is -inf, rejected for any t_max.
RT_D float coop_sphere_root(float4 s, const CoopRay &C, float tmin) {
  const f3 oc = sub(mk(C.ox, C.oy, C.oz), mk(s.x, s.y, s.z));
  const float b = dot(oc, mk(C.dx, C.dy, C.dz));
  const float c = dot(oc, oc) - s.w;
  const float disc = b * b - C.a * c;
  if (disc < 0) return -__builtin_inff();
  float sq = sqrt_core(disc);
  float q1 = div_core(-b - sq, C.a, C.ra), q2 = div_core(-b + sq, C.a, C.ra);
  const bool ok = (int)C.fast & ((int)(disc == 0.0f) | ((int)(disc >= kSqrtLo) & (int)(disc <= __FLT_MAX__))) &
                  (int)(fabsf(-b - sq) <= kNumHi) & (int)(fabsf(-b + sq) <= kNumHi);
  if (__builtin_expect(!ok, 0)) {
    sq = sqrtf(disc);
    q1 = (-b - sq) / C.a;
    q2 = (-b + sq) / C.a;
  }
  return (q1 <= tmin) ? q2 : q1;
}

// box entered at visit  <=>  !(fminf(t_max, X) <= E)  (E = fmaxf chain from t_min, X = fminf chain)
RT_D void box_interval(float4 q0, float4 q1, const CoopRay &C, float tmin, float &e, float &x) {
  const float t0x = (q0.x - C.ox) * C.ix, t1x = (q0.y - C.ox) * C.ix;
  const float t0y = (q0.z - C.oy) * C.iy, t1y = (q0.w - C.oy) * C.iy;
  const float t0z = (q1.x - C.oz) * C.iz, t1z = (q1.y - C.oz) * C.iz;
  const float nx = C.ix < 0 ? t1x : t0x, fx = C.ix < 0 ? t0x : t1x;
  const float ny = C.iy < 0 ? t1y : t0y, fy = C.iy < 0 ? t0y : t1y;
  const float nz = C.iz < 0 ? t1z : t0z, fz = C.iz < 0 ? t0z : t1z;
  e = fmaxf(fmaxf(fmaxf(tmin, nx), ny), nz);
  x = fminf(fminf(fx, fy), fz);
}

// The exact preorder scan with a whole wave: the wave evaluates a window of 64 consecutive items
// (box interval or sphere root, both t_max-independent), then scans it with wave-uniform decisions;
// a skip past the window, or its end, starts the next window.
RT_D void coop_trace9(const Book1View &V, const float4 *items, const CoopRay &C, float tmin, float &out_tmax,
                      int &out_hit) {
  const int lane = __lane_id();
  const int n = V.n_items9;
  float tmax = __builtin_inff();
  int hit = -1;
  int p = 0;
  int guard = 0;  // every scan step advances p, so n steps bound the walk; this only catches bugs
  while (p < n && guard <= n) {
    const int base = p;
    const int q = base + lane;
    float v0 = 0.0f, v1 = 0.0f;  // node: E, X; leaf: root
    uint32_t meta = 0;           // node: skip; leaf: index | kLeaf9
    if (q < n) {
      const float4 q0 = it_q0(items, q), q1 = it_q1(items, V.n_items9_alloc, q);
      meta = __float_as_uint(q1.w);
      if (meta & kLeaf9) {
        v0 = coop_sphere_root(q0, C, tmin);
      } else {
        box_interval(q0, q1, C, tmin, v0, v1);
        meta = __float_as_uint(q1.z);
      }
    }
    const int end = min(n, base + 64);
    // decisions for the current t_max in every lane, then a scalar walk along the next-pointers;
    // an accepted sphere changes t_max, so the decisions are redone from there
    const bool leaf = (meta & kLeaf9) != 0;
    const int l = lane;
    while (p < end && guard++ <= n) {
      const bool take = leaf ? !(v0 <= tmin || v0 >= tmax) : !(fminf(tmax, v1) <= v0);
      // next item after this one for the current t_max; an accepted sphere (t_max changes) is
      // encoded as kStop + its position so that the walk below only has to test one bound
      constexpr int kStop = 1 << 20;
      const int next = leaf ? (take ? kStop + l : l + 1) : (take ? l + 1 : l + (int)meta);
      const int wend = end - base;
      int at = p - base;
      while (at < wend) at = __builtin_amdgcn_readlane(next, at);
      if (at < kStop) {  // left the window
        p = base + at;
        break;
      }
      at -= kStop;  // an accepted sphere: t_max shrinks, the walk goes on after it
      tmax = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v0), at));
      hit = (int)((uint32_t)__builtin_amdgcn_readlane((int)meta, at) & kLeafIdx);
      p = base + at + 1;
    }
  }
  out_tmax = tmax;
  out_hit = hit;
}

// Closest hit by candidates.  The reference's traversal (preorder visit, box culling against the
// shrinking t_max) returns the first-visited sphere of least accepted root.  A sphere's accepted root
// r does not depend on t_max, so take s* = the leaf of least valid r (t_min < r < inf), earliest in
// preorder among equal r.  Every sphere visited before s* is earlier in preorder, so its root is
// > r*, and the t_max at each of s*'s ancestors' visits is > r*.  An ancestor box is then entered
// (monotone in t_max) whenever fminf(r*, X) > E; if that holds for all of s*'s ancestors, s* is
// visited, accepted and never displaced: the reference returns (r*, s*).  If the ancestor check
// fails (a grazing box) or a root is NaN, the exact scan (coop_trace9) runs.  A miss (no valid root
// at all) is exact: the reference cannot accept anything.
// Leaf n's item position is kept in a spare word of item n (q1.w of a node item, q1.x of a leaf
// item; host: book1_upload).  bf_candidate returns false (undecided: a NaN root) or the candidate
// (r*, p*), p* = -1 for a miss; bf_verify is the ancestor check of a candidate p* >= 0.
constexpr int kBfSlots = 8;  // 64 x 8 = 512 leaves at most (host-checked)

// Subtree cuts for the candidate trace (host: book1_pack): at most 64 subtrees that partition the leaves,
// each its root item q, its leaves [l0, l1) in preorder numbering and the node items enclosing q.  A
// subtree whose root box is not entered at t_max = +inf is never entered (the test is monotone in t_max:
// fminf(t, X) <= fminf(inf, X)), so none of its spheres is visited and none can be the reference's hit:
// the candidate trace evaluates the roots of the entered subtrees' spheres only, one per lane, and the
// ancestor check walks the cut's list and the cut's own subtree before the candidate.
constexpr int kBfAnc = 12;
struct BfCut {
  uint16_t q, l0, l1, n_anc;
  uint16_t anc[kBfAnc];
};

RT_D bool bf_candidate(const Book1View &V, const float4 *items, const CoopRay &C, float tmin, float &out_best,
                       int &out_bp) {
  const int lane = __lane_id();
  float best = __builtin_inff();
  int bp = 0x7fffffff;  // item position of the best leaf (preorder rank)
  bool nan = false;
  // (unrolled 4 / 8, or the slots' leaf positions or sphere words held in registers per work item:
  // same N = 1 and N = 8 times, same box, r04)
#pragma unroll 2
  for (int k = 0; k < kBfSlots; k++) {
    if (k * 64 >= V.n_bf_leaves) break;  // wave-uniform
    const int n = k * 64 + lane;
    const bool live = n < V.n_bf_leaves;
    const float4 h = it_q1(items, V.n_items9_alloc, live ? n : 0);
    const uint32_t hw = __float_as_uint(h.w);
    const int pos = (int)((hw & kLeaf9) ? __float_as_uint(h.x) : hw);
    const float r = coop_sphere_root(it_q0(items, pos), C, tmin);
    nan |= live && r != r;
    if (live && r > tmin && r < best) best = r, bp = pos;  // strict: the earlier slot wins ties
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {  // argmin over (root, preorder position)
    const float ob = __shfl_xor(best, off);
    const int op = __shfl_xor(bp, off);
    if (ob < best || (ob == best && op < bp)) best = ob, bp = op;
  }
  if (__ballot(nan) != 0) return false;
  out_best = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(best)));
  bp = __builtin_amdgcn_readfirstlane(bp);
  out_bp = bp == 0x7fffffff ? -1 : bp;  // no valid root anywhere: a miss
  return true;
}

RT_D bool bf_verify(const float4 *items, int na, const CoopRay &C, float tmin, float best, int bp) {
  const int lane = __lane_id();
  bool bad = false;
  for (int base = 0; base < bp; base += 64) {  // wave-uniform bound
    const int q = base + lane;
    if (q < bp) {
      const float4 q1 = it_q1(items, na, q);
      const uint32_t w = __float_as_uint(q1.w);
      if (!(w & kLeaf9) && (uint32_t)bp < (uint32_t)q + __float_as_uint(q1.z)) {  // an ancestor of p*
        float e, x;
        box_interval(it_q0(items, q), q1, C, tmin, e, x);
        bad |= !(fminf(best, x) > e);
      }
    }
  }
  return __ballot(bad) == 0;
}

// Wave scans on DPP (row shifts within 16-lane rows, then the gfx9 row broadcasts of lanes 15 and 31)
// instead of ds_bpermute: a step is a VALU move, not an LDS-crossbar round trip.  Every lane must be
// active.  Lanes without a source keep `old`, the operation's identity.
constexpr int kDppRowShr = 0x110, kDppBcast15 = 0x142, kDppBcast31 = 0x143;
template <int kCtrl, int kRows>
RT_D uint32_t dpp_mov(uint32_t old, uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, kCtrl, kRows, 0xf, false);
}
template <int kCtrl, int kRows>
RT_D void dpp_sum_step(uint32_t &x) { x += dpp_mov<kCtrl, kRows>(0u, x); }
RT_D uint32_t wave_incl_sum(uint32_t x) {  // inclusive prefix sum over the lanes
  dpp_sum_step<kDppRowShr + 1, 0xf>(x);
  dpp_sum_step<kDppRowShr + 2, 0xf>(x);
  dpp_sum_step<kDppRowShr + 4, 0xf>(x);
  dpp_sum_step<kDppRowShr + 8, 0xf>(x);
  dpp_sum_step<kDppBcast15, 0xa>(x);  // rows 1, 3 += lane 15 / 47
  dpp_sum_step<kDppBcast31, 0xc>(x);  // rows 2, 3 += lane 31
  return x;
}
template <int kCtrl, int kRows>
RT_D void dpp_max_step(uint32_t &x) {
  const uint32_t o = dpp_mov<kCtrl, kRows>(0u, x);
  x = o > x ? o : x;
}
RT_D uint32_t wave_incl_max(uint32_t x) {  // inclusive prefix max over the lanes
  dpp_max_step<kDppRowShr + 1, 0xf>(x);
  dpp_max_step<kDppRowShr + 2, 0xf>(x);
  dpp_max_step<kDppRowShr + 4, 0xf>(x);
  dpp_max_step<kDppRowShr + 8, 0xf>(x);
  dpp_max_step<kDppBcast15, 0xa>(x);
  dpp_max_step<kDppBcast31, 0xc>(x);
  return x;
}
template <int kCtrl, int kRows>
RT_D void dpp_min_step(uint64_t &k) {
  const uint32_t lo = dpp_mov<kCtrl, kRows>(0xffffffffu, (uint32_t)k);
  const uint32_t hi = dpp_mov<kCtrl, kRows>(0xffffffffu, (uint32_t)(k >> 32));
  const uint64_t o = (uint64_t)hi << 32 | lo;
  k = o < k ? o : k;
}
RT_D uint64_t wave_min_u64(uint64_t k) {  // the least key of the wave (wave-uniform)
  dpp_min_step<kDppRowShr + 1, 0xf>(k);
  dpp_min_step<kDppRowShr + 2, 0xf>(k);
  dpp_min_step<kDppRowShr + 4, 0xf>(k);
  dpp_min_step<kDppRowShr + 8, 0xf>(k);
  dpp_min_step<kDppBcast15, 0xa>(k);
  dpp_min_step<kDppBcast31, 0xc>(k);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)k, 63);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(k >> 32), 63);
  return (uint64_t)hi << 32 | lo;
}

// bf_candidate on the entered subtrees only (BfCut above); cut = the candidate's subtree (for bf_verify_cut).
RT_D bool bf_candidate_cut(const Book1View &V, const float4 *items, const CoopRay &C, float tmin, float &out_best,
                           int &out_bp, int &out_cut) {
  const int lane = __lane_id();
  const bool has = lane < V.n_bf_cuts;
  uint32_t l0 = 0, cnt = 0;
  if (has) {
    const BfCut &K = V.bf_cuts[lane];
    const float4 q1 = it_q1(items, V.n_items9_alloc, K.q);
    bool in = true;  // a single sphere: always a candidate
    if (!(__float_as_uint(q1.w) & kLeaf9)) {
      float e, x;
      box_interval(it_q0(items, K.q), q1, C, tmin, e, x);
      in = !(fminf(__builtin_inff(), x) <= e);
    }
    l0 = K.l0;
    cnt = in ? (uint32_t)(K.l1 - K.l0) : 0u;
  }
  const uint32_t incl = wave_incl_sum(cnt);
  const uint32_t excl = incl - cnt;
  const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
  // a non-empty cut's key: its index and the offset from its compacted leaves to its leaf numbers
  // (l0 >= excl: compaction only drops leaves), so that a lane's leaf is g + offset
  const uint32_t ckey = (uint32_t)lane << 16 | (l0 - excl);
  const uint64_t nonempty = __ballot(cnt > 0);
  float best = __builtin_inff();
  int bp = 0x7fffffff, bc = -1;
  bool nan = false;
  for (uint32_t base = 0; base < total; base += 64) {  // wave-uniform
    const uint32_t g = base + (uint32_t)lane;
    // the lane's subtree: the last non-empty one starting at or before g.  Its key is written to the lane
    // where it starts (lane 0: the cut that holds `base`; a scalar loop over the cuts
    // that start inside the window), then a prefix max hands every lane the last start before it (the
    // keys grow with the start).
    const uint64_t upto = nonempty & __ballot(excl <= base);  // (non-empty: holds the cut of excl 0)
    const int c0 = 63 - (int)__builtin_clzll(upto);
    uint32_t mark = lane == 0 ? (uint32_t)__builtin_amdgcn_readlane((int)ckey, c0) : 0u;
    for (uint64_t st = nonempty & __ballot(excl > base && excl < base + 64u); st; st &= st - 1) {
      const int c = (int)__builtin_ctzll(st);
      const int at = __builtin_amdgcn_readlane((int)excl, c) - (int)base;
      const uint32_t kc = (uint32_t)__builtin_amdgcn_readlane((int)ckey, c);
      mark = lane == at ? kc : mark;
    }
    const uint32_t k = wave_incl_max(mark);
    const int c = (int)(k >> 16);
    const bool live = g < total;
    const int n = live ? (int)(g + (k & 0xffffu)) : 0;
    const float4 h = it_q1(items, V.n_items9_alloc, n);
    const uint32_t hw = __float_as_uint(h.w);
    const int pos = (int)((hw & kLeaf9) ? __float_as_uint(h.x) : hw);
    const float r = coop_sphere_root(it_q0(items, pos), C, tmin);
    nan |= live && r != r;
    if (live && r > tmin && (r < best || (r == best && pos < bp))) best = r, bp = pos, bc = c;
  }
  // argmin over (root, preorder position): a valid root is > t_min > 0, so its bits order as the floats
  const uint64_t key = (uint64_t)__float_as_uint(best) << 32 | (uint32_t)bp;
  const uint64_t win = wave_min_u64(key);
  if (__ballot(nan) != 0) return false;
  const int wl = __builtin_amdgcn_readfirstlane(__ffsll((unsigned long long)__ballot(key == win)) - 1);
  out_best = __uint_as_float((uint32_t)(win >> 32));
  bp = (int)(uint32_t)win;
  out_cut = __builtin_amdgcn_readlane(bc, wl);
  out_bp = bp == 0x7fffffff ? -1 : bp;  // no valid root in any entered subtree: a miss
  return true;
}

// bf_verify for a candidate of subtree cut: its ancestors are the cut's list and the nodes of the cut's
// own subtree (its root included) that enclose bp.
RT_D bool bf_verify_cut(const Book1View &V, const float4 *items, const CoopRay &C, float tmin, float best, int bp,
                        int cut) {
  const int lane = __lane_id();
  const int na = V.n_items9_alloc;
  const BfCut &K = V.bf_cuts[cut];
  const int n_anc = K.n_anc;
  bool bad = false;
  {  // one pass: lanes [0, n_anc) the cut's ancestors, the lanes above them the cut's first items before bp
    const int q = lane < n_anc ? (int)K.anc[lane] : (int)K.q + (lane - n_anc);
    if (q < bp) {  // (an ancestor precedes bp)
      const float4 q1 = it_q1(items, na, q);
      const uint32_t w = __float_as_uint(q1.w);
      if (lane < n_anc || (!(w & kLeaf9) && (uint32_t)bp < (uint32_t)q + __float_as_uint(q1.z))) {
        float e, x;
        box_interval(it_q0(items, q), q1, C, tmin, e, x);
        bad = !(fminf(best, x) > e);
      }
    }
  }
  for (int base = (int)K.q + 64 - n_anc; base < bp; base += 64) {  // wave-uniform bound (rarely entered)
    const int q = base + lane;
    if (q < bp) {
      const float4 q1 = it_q1(items, na, q);
      const uint32_t w = __float_as_uint(q1.w);
      if (!(w & kLeaf9) && (uint32_t)bp < (uint32_t)q + __float_as_uint(q1.z)) {  // an ancestor of p*
        float e, x;
        box_interval(it_q0(items, q), q1, C, tmin, e, x);
        bad |= !(fminf(best, x) > e);
      }
    }
  }
  return __ballot(bad) == 0;
}

// The record arena is clean (every record's end word kRecFill) between chain launches: a chain launch
// reserves and may write records [0, n) (n: chain_plan_kernel's reservations), and the next launch's
// cost pre-pass sets them back, in the waves that have run out of pixels -- at N >= 2 most of the
// pre-pass's waves idle from the start (0.4 pixels per lane at N = 8), so the 4-5 GB of a share's
// reservation are written while the pre-pass's heaviest pixels run instead of after the plan (the
// chain_fill_kernel of r01-r05: 0.9 ms per N = 8 share).  Claims of kCleanChunk records per wave.
constexpr uint32_t kCleanChunk = 16384;
__attribute__((noinline)) RT_D void clean_records(float4 *col, const uint32_t *n_p, unsigned long long *ctr) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint64_t n = *n_p;
  const int lane = __lane_id();
  const float4 fill = make_float4(0.0f, 0.0f, 0.0f, u2f(kRecFill));
  for (;;) {
    unsigned long long c0 = 0;
    if (lane == 0) c0 = atomicAdd(ctr, (unsigned long long)kCleanChunk);
    c0 = __shfl(c0, 0);
    if (c0 >= n) return;
    const uint64_t c1 = c0 + kCleanChunk < n ? c0 + kCleanChunk : n;
    for (uint64_t i = c0 + (uint64_t)lane; i < c1; i += 64) col[i] = fill;
  }
#endif
}

// ---------------------------------------------------------------- chain protocol (kMode 2)
// Coupling cursor: successor segment t << 24 | record c.
constexpr uint32_t kCurRec = 0xffffffu;

// Coupling scan of chain k at its sample boundary x: does a successor record start at x?  tc = the
// cursor, st = the start offset of its record.  Returns true when coupled (tc then names the record
// that starts at x).  Bounded work per call; a record not yet written, or a successor still running
// past its last record, is looked at again next time.
RT_D bool chain_couple(const Book1View &V, const ChainPx &P, uint32_t k, uint32_t x, uint32_t &tc, uint32_t &st) {
  for (int it = 0; it < 24; it++) {
    const uint32_t t = tc >> 24, c = tc & kCurRec;
    if (t >= P.K) return false;  // no successor (kNoTarget)
    if (st > x) return false;  // the successor's next sample starts beyond x
    if (st == x) return true;
    if (c < seg_cap(P, t)) {  // st < x: step over record c
      const uint32_t e = rec_end(V, rec_index(P, t, c));
      if (e != kRecFill) {
        st = e;
        tc = (tc & ~kCurRec) | (c + 1u);
        continue;
      }
    }
    // record c is not there (yet): follow the successor's link if it has ended past its last record
    const uint64_t w = ld_rel64(&V.ch_seg[P.end0 + t]);
    if (!(w & kEndEnded) || c < end_n(w)) return false;  // running, or its record c still in flight
    if (w & kEndNoLink) {
      tc = kNoTarget;  // it ended without a link: nothing to couple with beyond it
      return false;
    }
    const uint32_t t2 = end_t(w), c2 = end_c(w);
    if (t2 <= t || t2 >= P.K) {  // (never: links point forward)
      tc = kNoTarget;
      return false;
    }
    uint32_t s2 = seg_start(P, t2);
    if (c2 > 0) {
      s2 = rec_end(V, rec_index(P, t2, c2 - 1u));
      if (s2 == kRecFill) return false;
    }
    tc = (t2 << 24) | c2;
    st = s2;
  }
  return false;
}

// Does chain k (holding n records) still have work?  Follows the links from segment 0: returns true
// (stop) when the pixel's spp true samples are already covered up to this chain's records, or when
// the true chain provably never reaches this chain (it jumps past k's start); false while undecided.
RT_D bool chain_walk_done(const Book1View &V, const ChainPx &P, uint32_t k, uint32_t n, uint32_t spp) {
  uint64_t w = ld_rel64(&V.ch_seg[P.end0]);
  if (!(w & kEndEnded)) return false;
  if (w & kEndNoLink) return true;  // segment 0 completed the pixel
  uint32_t total = end_n(w), t = end_t(w), c = end_c(w);
  for (uint32_t it = 0; it < P.K; it++) {
    if (t == k) return total + (n - c) >= spp;
    if (t > k) return true;  // the true chain skips this chain
    w = ld_rel64(&V.ch_seg[P.end0 + t]);
    if (!(w & kEndEnded)) return false;
    if (w & kEndNoLink) return true;  // the true chain ends (or breaks) before this chain
    total += end_n(w) - c;
    if (total >= spp) return true;
    t = end_t(w), c = end_c(w);
  }
  return false;
}

// A chain's sample boundary (kMode 2): before each sample.  seg = the item's segment word; s = the
// true samples taken (segment 0, unsplit, continuation) or the records written (segment >= 1);
// x = the stream offset.  Returns true when the work item is finished (pixel written or end word
// stored).  writer: this lane stores (false in the lanes of a wave-uniform caller other than lane 0).
RT_D bool chain_boundary_(const Book1View &V, int64_t pix, uint32_t seg, uint32_t x, uint32_t s, f3 acc,
                          uint32_t &tc, uint32_t &st, uint8_t *__restrict__ out, bool writer);
// (diagnostic timeline, RT_PX_TIME=1: a chain's start and end in wall_clock64 ticks)
// (word 3: where the item started -- XCC_ID << 28 | HW_ID's wave, SIMD, pipe, CU, SH and SE fields)
constexpr int kTimeWords = 4;
RT_D uint32_t hw_where() {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t hw = __builtin_amdgcn_s_getreg(4 | (31 << 11));      // HW_REG_HW_ID, 32 bits
  const uint32_t xcc = __builtin_amdgcn_s_getreg(20 | (3 << 11));     // HW_REG_XCC_ID, 4 bits
  return (xcc << 28) | (hw & 0xffffu);
#else
  return 0u;
#endif
}
RT_D void chain_time(const Book1View &V, int64_t pix, uint32_t seg, int end) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t now = (uint32_t)wall_clock64();
  uint32_t *w = (seg & kItemUnsplit) ? V.px_time + kTimeWords * pix : V.seg_time + kTimeWords * (V.ch_px[pix].end0 + seg);
  w[end] = now;
  if (end == 0) w[3] = hw_where();
#endif
}
RT_D bool chain_boundary(const Book1View &V, int64_t pix, uint32_t seg, uint32_t x, uint32_t s, f3 acc,
                         uint32_t &tc, uint32_t &st, uint8_t *__restrict__ out, bool writer) {
  const bool done = chain_boundary_(V, pix, seg, x, s, acc, tc, st, out, writer);
  if (done && writer && V.px_time) chain_time(V, pix, seg, 1);
  return done;
}
RT_D bool chain_boundary_(const Book1View &V, int64_t pix, uint32_t seg, uint32_t x, uint32_t s, f3 acc,
                          uint32_t &tc, uint32_t &st, uint8_t *__restrict__ out, bool writer) {
  const uint32_t spp = (uint32_t)V.S.cam.spp;
  if (seg & kItemUnsplit) {  // the whole pixel (or a continuation)
    if (s < spp) return false;
    if (writer) write_pixel(out + pix * 3, acc, (int)spp);
    return true;
  }
  const ChainPx P = V.ch_px[pix];
  const uint32_t k = seg;
  if (k == 0 && s >= spp) {  // the head reached the end before coupling
    if (writer) {
      write_pixel(out + pix * 3, acc, (int)spp);
      st_rel64(&V.ch_seg[P.end0], end_word(s, false, 0u));
    }
    return true;
  }
  if (k > 0 && s >= seg_cap(P, k)) {  // the list is full
    if (writer) st_rel64(&V.ch_seg[P.end0 + k], end_word(s, false, 0u));
    return true;
  }
  if (chain_couple(V, P, k, x, tc, st)) {
    if (writer) {
      if (k == 0) V.ch_acc0[pix] = make_float4(acc.x, acc.y, acc.z, 0.0f);
      st_rel64(&V.ch_seg[P.end0 + k], end_word(s, true, tc));
    }
    return true;
  }
  if (k > 0 && s >= P.check && (s & V.walk_mask) == 0u && chain_walk_done(V, P, k, s, spp)) {
    if (writer) st_rel64(&V.ch_seg[P.end0 + k], end_word(s, false, 0u));
    return true;
  }
  return false;
}

// Record of a segment >= 1 chain: the sample's colour and end offset (g.n after it), one 16-B
// write-through store (the coupling scans of other chains read its end word while the launch runs,
// the fold its colour after it).
RT_D void chain_record(const Book1View &V, int64_t pix, uint32_t k, uint32_t c, f3 col, uint32_t x_end) {
  const ChainPx &P = V.ch_px[pix];
  st_rel128(&V.ch_col[rec_index(P, k, c)], make_float4(col.x, col.y, col.z, u2f(x_end)));
}

// A chain's start: stream position, and its coupling cursor on its successor.
RT_D void chain_start(const Book1View &V, uint32_t pix, uint32_t seg, Pcg32 &g, uint32_t &tc, uint32_t &st) {
  const ChainPx &P = V.ch_px[pix];
  g.skip(seg_start(P, seg));
  const uint32_t n = seg_next(P, seg);
  tc = n << 24;  // (kNone << 24 == kNoTarget)
  st = n == kNone ? 0u : seg_start(P, n);
}

// ---------------------------------------------------------------- whole-wave work items
// A work item rendered by one wave: the path state is wave-uniform (every lane holds the same
// values and runs the same shading), and each ray is traced by the wave (bf_candidate + bf_verify,
// or the exact scan).  The item is a whole pixel (kMode 0: its samples in order), or a chain
// (kMode 2: segment / unsplit pixel, with the same boundary protocol as a lane).
template <int kMode>
RT_D void render_item_coop(const Book1View &V, const float4 *items9, int64_t pix, uint32_t seg,
                           uint8_t *__restrict__ out, const MigRec *res = nullptr) {
  const rt_camera &cam = V.S.cam;
  const int W = cam.width;
  const int jj = (int)(pix / W);
  const int i = (int)(pix - (int64_t)jj * W);
  const int j = V.row0 + jj * V.row_stride;
  const f3 du = ld3(cam.delta_u), dv = ld3(cam.delta_v), lf = ld3(cam.origin);
  const float tmin = 1e-3f;
  const bool lane0 = __lane_id() == 0;
  Pcg32 g;
  g.seed((uint64_t)(17 + j), (uint64_t)(23 + i));  // src/raytracing.c:94
  f3 acc = mk(0.0f, 0.0f, 0.0f);
  uint32_t s = 0, tc = kNoTarget, st = 0;
  if (res) {  // a migrated item: on from the lane's sample boundary
    g.state = res->state;
    g.n = res->n;
    s = res->s, tc = res->tc, st = res->st;
    acc = mk(res->acc[0], res->acc[1], res->acc[2]);
  } else if (kMode == 2) {
    if (!(seg & kItemUnsplit)) chain_start(V, (uint32_t)pix, seg, g, tc, st);
    pre_resume(V, pix, seg, g, s, acc);
  }
  const bool use_bf = V.n_bf_leaves > 0;
  const uint32_t px_start = V.px_time && !res ? (uint32_t)wall_clock64() : 0u;
  if (kMode == 2 && V.px_time && lane0 && !res) chain_time(V, pix, seg, 0);
#ifdef RT_DIAG
  // (diagnostic: a migrated item's rays, exact scans, and shader clocks in the candidate trace, the
  // ancestor check, the exact scans and the whole item)
  uint64_t d_ray = 0, d_exact = 0, d_cand = 0, d_ver = 0, d_scan = 0;
  const uint64_t d_t0 = clock64();
#endif
  for (;;) {
    if (kMode == 2) {  // (wave-uniform: every lane loads the same words; lane 0's view decides)
      const bool done = chain_boundary(V, pix, seg, g.n, s, acc, tc, st, out, lane0);
      tc = (uint32_t)__builtin_amdgcn_readfirstlane((int)tc);
      st = (uint32_t)__builtin_amdgcn_readfirstlane((int)st);
      if (__builtin_amdgcn_readfirstlane((int)done)) break;
    } else if (s == (uint32_t)cam.spp) {
      break;
    }
    // camera ray (src/raytracing.c:96-122)
    const f3 pixel_pos = add(add(ld3(cam.pixel00), scale(du, (float)i)), scale(dv, (float)j));
    const float px = g.between(-0.5f, 0.5f);
    const float py = g.between(-0.5f, 0.5f);
    f3 o = lf;
    if (cam.dof_angle > 0.0f) {
      float a, b;
      for (;;) {
        a = g.between(-1.0f, 1.0f);
        b = g.between(-1.0f, 1.0f);
        if (a * a + b * b < 1.0f) break;
      }
      o = add(add(lf, scale(ld3(cam.disc_u), a)), scale(ld3(cam.disc_v), b));
    }
    f3 d = add(add(add(pixel_pos, scale(du, px)), scale(dv, py)), neg(o));
    // the path record lives in the lanes: lane k holds the albedo of bounce k (max_depth <= 64,
    // book1_eligible), folded with readlane instead of a chain of material loads
    float ar = 0.0f, ag = 0.0f, ab = 0.0f;
    int n_b = 0;
    f3 tail = mk(0.0f, 0.0f, 0.0f);
    for (int depth = cam.max_depth; depth > 0;) {  // Camera_ray_color (src/raytracing.c:39-75)
      CoopRay C;
      C.ox = o.x, C.oy = o.y, C.oz = o.z, C.dx = d.x, C.dy = d.y, C.dz = d.z;
      C.ix = 1.0f / d.x, C.iy = 1.0f / d.y, C.iz = 1.0f / d.z;
      C.a = dot(d, d);
      C.fast = C.a >= kDivLo && C.a <= kDivHi;
      C.ra = recip_core(C.a);
      float tmax = __builtin_inff();
      int bp = -1, cut = -1;
#ifdef RT_DIAG
      const uint64_t d_a = clock64();
#endif
      bool decided = use_bf && (V.n_bf_cuts > 0 ? bf_candidate_cut(V, items9, C, tmin, tmax, bp, cut)
                                                : bf_candidate(V, items9, C, tmin, tmax, bp));
#ifdef RT_DIAG
      const uint64_t d_b = clock64();
      d_cand += d_b - d_a, d_ray++;
#endif
      // the hit sphere (center, 1/r, material) from its LDS item, and its material's load issued
      // before the ancestor check so that its latency overlaps it
      float4 s0 = make_float4(0.0f, 0.0f, 0.0f, 0.0f), s1 = s0;
      FastMat m;
      if (decided && bp >= 0) {
        s0 = it_q0(items9, bp), s1 = it_q1(items9, V.n_items9_alloc, bp);
        m = V.mats[__float_as_int(s1.z)];
        decided = V.n_bf_cuts > 0 ? bf_verify_cut(V, items9, C, tmin, tmax, bp, cut)
                                  : bf_verify(items9, V.n_items9_alloc, C, tmin, tmax, bp);
#ifdef RT_DIAG
        d_ver += clock64() - d_b;
#endif
      }
      if (!decided) {  // the exact scan
        int hit;
#ifdef RT_DIAG
        const uint64_t d_c = clock64();
#endif
        coop_trace9(V, items9, C, tmin, tmax, hit);
#ifdef RT_DIAG
        d_scan += clock64() - d_c, d_exact++;
#endif
        bp = hit;
        if (hit >= 0) {
          const rt_sphere &sp = V.S.spheres[hit];
          s0 = make_float4(sp.center[0], sp.center[1], sp.center[2], 0.0f);
          s1 = make_float4(0.0f, sp.inv_radius, __int_as_float(sp.material), 0.0f);
          m = V.mats[sp.material];
        }
      }
      if (bp < 0) {
        tail = ld3(cam.background);
        break;
      }
      const f3 p = ray_at(o, d, tmax);
      const f3 outward = scale(sub(p, mk(s0.x, s0.y, s0.z)), s1.y);
      const bool front = dot(d, outward) < 0.0f;
      const f3 normal = front ? outward : neg(outward);
      const f3 nd = scatter(m, normal, front, d, g);
      if (__lane_id() == n_b) ar = m.albedo[0], ag = m.albedo[1], ab = m.albedo[2];
      n_b++;
      o = p;
      d = nd;
      depth--;
    }
    f3 c = tail;  // fold innermost first, as the recursion returns: c = 0 + a_k (x) c (rec_fold_chunk)
    for (int k = n_b - 1; k >= 0; k--) {
      const f3 a = mk(lane_bcast(ar, k), lane_bcast(ag, k), lane_bcast(ab, k));
      c = add(mk(0.0f, 0.0f, 0.0f), mul(a, c));
    }
    if (kMode == 2 && !(seg & kItemUnsplit) && seg > 0) {
      if (lane0) chain_record(V, pix, seg, s, c, g.n);
    } else {
      acc = add(acc, c);
    }
    s++;
  }
#ifdef RT_DIAG
  if (res && V.px_time && lane0) {
    unsigned long long *st = (unsigned long long *)(V.mig + kMigStat);
    atomicAdd(st + 0, (unsigned long long)d_ray), atomicAdd(st + 1, (unsigned long long)d_exact);
    atomicAdd(st + 2, (unsigned long long)d_cand), atomicAdd(st + 3, (unsigned long long)d_ver);
    atomicAdd(st + 4, (unsigned long long)d_scan), atomicAdd(st + 5, (unsigned long long)(clock64() - d_t0));
  }
#endif
  if (kMode != 2 && lane0) write_pixel(out + pix * 3, acc, cam.spp);
  if (V.px_time && lane0 && kMode != 2) {
    if (!res) V.px_time[kTimeWords * pix] = px_start;
    V.px_time[kTimeWords * pix + 1] = (uint32_t)wall_clock64();
  }
}

// ---------------------------------------------------------------- migration (MigRec)
RT_D uint32_t *mig_box(const Book1View &V, uint32_t m) { return V.mig + kMigBox0 + m * kMigBoxWords; }

// An item finished (in a lane or a helper): the last one tells every mailbox.
RT_D void mig_item_done(const Book1View &V, int64_t total_own) {
  if ((int64_t)atomicAdd(&V.mig[kMigDone], 1u) + 1 == total_own)
    for (int m = 0; m < kMigBoxes; m++) st_rel(mig_box(V, (uint32_t)m) + kMigFinished, 1u);
}

RT_D bool mig_push(const Book1View &V, uint32_t m, int32_t pix, uint32_t seg, uint32_t s, f3 acc, const Pcg32 &g,
                   uint32_t tc, uint32_t st) {
  uint32_t *box = mig_box(V, m);
  if ((int32_t)atomicSub(box + kMigCredits, 1u) <= 0) {  // no idle helper here: keep the item
    atomicAdd(box + kMigCredits, 1u);
    return false;
  }
  const uint32_t cap = V.mig_cap / kMigBoxes;
  const uint32_t idx = atomicAdd(box + kMigPush, 1u);
  if (idx >= cap) {  // this mailbox's queue is full (its helpers never look past cap)
    atomicAdd(box + kMigCredits, 1u);
    return false;
  }
  MigRec &r = V.mig_q[m * cap + idx];
  r.state = g.state;
  r.n = g.n;
  r.pix = (uint32_t)pix, r.seg = seg, r.s = s, r.tc = tc, r.st = st;
  r.acc[0] = acc.x, r.acc[1] = acc.y, r.acc[2] = acc.z;
  __hip_atomic_store(&r.ready, V.mig_epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  return true;
}

// The scene items of the whole-wave traces in the (not inlined) helper functions: a pointer derived
// from the LDS symbol itself, so that their loads compile to ds_read (a pointer passed in as a
// parameter is generic there: flat loads, which wait on both the memory and the LDS counters).
template <bool kLds>
__device__ __forceinline__ const float4 *items9_of(const Book1View &V) {
  extern __shared__ __attribute__((aligned(16))) char rt_items_lds[];
  return kLds ? (const float4 *)rt_items_lds : (const float4 *)V.items9_g;
}
// The launch's view in the helper functions: the kernel argument segment's address, passed as a
// constant-address-space pointer (a generic reference would make every field read a flat load
// instead of a scalar one; a callee's own __builtin_amdgcn_kernarg_segment_ptr() is null).
typedef const __attribute__((address_space(4))) Book1View *KernargView;
__device__ __forceinline__ KernargView kernarg_view() {
#if defined(__HIP_DEVICE_COMPILE__)
  return (KernargView)__builtin_amdgcn_kernarg_segment_ptr();
#else
  return nullptr;
#endif
}
// (a pointer argument arrives in VGPRs: made wave-uniform again, the field reads are scalar loads)
__device__ __forceinline__ const Book1View &view_of(KernargView kv) {
  const uint64_t a = (uint64_t)kv;
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)a);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(a >> 32));
  return *(const Book1View *)(KernargView)(((uint64_t)hi << 32) | lo);
}

#ifndef RT_HELP_PRIO
#define RT_HELP_PRIO 2
#endif
// A wave whose lanes have all finished: run the migrated items of its mailbox until every item of
// the launch is done.
template <int kMode, bool kLds>
__device__ __attribute__((noinline)) void mig_help(KernargView kv, uint8_t *__restrict__ out, int64_t total_own) {
  const Book1View &V = view_of(kv);
  const float4 *items9 = items9_of<kLds>(V);
  const bool l0 = __lane_id() == 0;
  const uint32_t wave = (blockIdx.x * kBlock + threadIdx.x) / 64;
  const uint32_t m = wave % kMigBoxes;
  uint32_t *box = mig_box(V, m);
  const uint32_t cap = V.mig_cap / kMigBoxes;
  int rank = 0;
  if (l0) rank = (int)atomicAdd(&V.mig[kMigHelpers], 1u);  // waves finished before this one
  rank = __builtin_amdgcn_readfirstlane(rank);
  if (rank >= V.mig_max_help) return;  // enough helpers: this wave leaves (its CU may idle)
  if (l0) atomicAdd(box + kMigCredits, 1u);
  uint64_t idle_since = wall_clock64();
  for (;;) {
    int got = -1, fin = 0;
    if (l0) {
      const uint32_t p = ld_rel(box + kMigPop);
      uint32_t q = ld_rel(box + kMigPush);
      fin = (int)ld_rel(box + kMigFinished);
      q = q < cap ? q : cap;
      if (p < q && atomicCAS(box + kMigPop, p, p + 1u) == p) got = (int)p;
    }
    got = __builtin_amdgcn_readfirstlane(got);
    if (got >= 0) {
      const MigRec *q = &V.mig_q[m * cap + (uint32_t)got];
      while (__hip_atomic_load(&q->ready, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) != V.mig_epoch)
        __builtin_amdgcn_s_sleep(1);
      MigRec r = *q;
      r.pix = (uint32_t)__builtin_amdgcn_readfirstlane((int)r.pix);
      r.seg = (uint32_t)__builtin_amdgcn_readfirstlane((int)r.seg);
      if (V.px_time && l0 && kMode == 2) chain_time(V, r.pix, r.seg, 2);  // (diagnostic: when it migrated)
      int drop = 0;
#ifdef RT_DIAG
      // (fault injection, diagnostic build only: drop the item unrun and uncounted -- chain_check_kernel
      // must then report the launch as incomplete)
      if (V.mig_drop && l0) drop = atomicAdd(&V.mig[kMigDropped], 1u) < V.mig_drop;
#endif
      if (!__builtin_amdgcn_readfirstlane(drop)) {
        __builtin_amdgcn_s_setprio(RT_HELP_PRIO);  // the frame's last chains: issue ahead of the lanes' waves
        render_item_coop<kMode>(V, items9, (int64_t)r.pix, r.seg, out, &r);
        __builtin_amdgcn_s_setprio(0);
        if (l0) mig_item_done(V, total_own);
      }
      if (l0) atomicAdd(box + kMigCredits, 1u);
      idle_since = wall_clock64();
      continue;
    }
    if (__builtin_amdgcn_readfirstlane(fin)) break;
    // A helper idle for mig_wait leaves -- but only by taking back a credit that no push has claimed.
    // A claimed credit stands for an item that is (being) queued in this mailbox, which then still
    // has a helper to run it; so no item is ever queued to a mailbox whose helpers have all left.
    // (Every item done sets kMigFinished; the bound only frees CU slots in long tails.)
    if (wall_clock64() - idle_since > V.mig_wait) {
      int left = 0;
      if (l0) {
        uint32_t c = ld_rel(box + kMigCredits);
        while ((int32_t)c > 0) {
          const uint32_t prev = atomicCAS(box + kMigCredits, c, c - 1u);
          if (prev == c) {
            left = 1;
            break;
          }
          c = prev;
        }
      }
      if (__builtin_amdgcn_readfirstlane(left)) break;
    }
    for (int k = 0; k < V.mig_sleep; k++) __builtin_amdgcn_s_sleep(127);  // ~3.4 us each
  }
}

// A chain launch's whole-wave items (the first *n_coop of ch_items), claimed one per wave through
// coop_counter by the chain kernel's first *coop_waves_dev waves.  Not inlined (see mig_help).
template <bool kLds>
__device__ __attribute__((noinline)) void coop_items(KernargView kv, uint8_t *__restrict__ out) {
  const Book1View &V = view_of(kv);
  const float4 *items9 = items9_of<kLds>(V);
  const int64_t n_coop = (int64_t)*V.n_coop;
  for (;;) {
    int k = 0;
    if (__lane_id() == 0) k = atomicAdd(V.coop_counter, 1);
    k = __shfl(k, 0);
    if (k >= n_coop) break;
    __builtin_amdgcn_s_setprio(3);  // these chains set the frame time: issue before the lane-parallel waves
    const uint2 it = V.ch_items[k];
    render_item_coop<2>(V, items9, (int64_t)it.x, it.y, out);
    __builtin_amdgcn_s_setprio(0);
  }
}

enum : int { kTrav = 0, kWait = 1, kExit = 2 };
// Issue priority of a chain launch's lane waves by their live lanes (r06): until the work
// items run out every wave is full (a lane that finishes an item takes the next in the same pass); after
// that the waves that still hold the most chains -- where the launch's last ones are -- issue first on
// their SIMD.  RT_LIVE_PRIO=0 (compile time): off, for A/B builds.
#ifndef RT_LIVE_PRIO
#define RT_LIVE_PRIO 1
#endif// traversal steps per pass before the wave re-checks its shading batch (measured, N = 1 kernel:
// 3: 384 ms, 4: 362 ms, 6: 345 ms, 8: 334 ms, 12: 330 ms, 16: 324 ms; frames identical -- the
// schedule never changes a lane)
constexpr int kSteps = 16;

// The lane kernel.  kMode: 0 frame (whole pixels), 1 cost pre-pass (also counts draws per item),
// 2 chain render (items of ch_items, or the continuation items of ch_cont).
template <bool kLds, int kMode = 0>
__device__ void render_batched(const Book1View &V, uint8_t *__restrict__ out, char *lds) {
  const int tid = threadIdx.x;
  const bool cont = kMode == 2 && V.ch_cont != nullptr;
  if (cont && *V.ch_n_cont == 0u) return;  // (before staging the scene: the usual continuation launch is empty)
  const int W = V.S.cam.width;
  const int64_t total = (int64_t)V.n_rows * W;
  float4 *items9 = (float4 *)lds;
  if (kLds) {
    for (int q = tid; q < 2 * V.n_items9_alloc; q += kBlock) items9[q] = V.items9_g[q];
    __syncthreads();
  } else {
    items9 = (float4 *)V.items9_g;
  }
  const int glane = blockIdx.x * kBlock + tid;
  const int lane = __lane_id();
  if (kMode == 2 && V.n_coop != nullptr && glane / 64 < (int)*V.coop_waves_dev) {
    // the chain launch's whole-wave items (heaviest first), in this kernel's first waves: a second
    // kernel next to this one got its CU slots only once workgroups of this one had finished
    // (measured: whole-wave items starting at 64 ms of a 106-ms launch); then on to lane items
    coop_items<kLds>(kernarg_view(), out);
  }
  const rt_camera &cam = V.S.cam;
  const f3 du = ld3(cam.delta_u), dv = ld3(cam.delta_v), lf = ld3(cam.origin);
  const bool dof = cam.dof_angle > 0.0f;
  const int spp = cam.spp, max_depth = cam.max_depth;
  const float tmin = 1e-3f;

  int mode = kWait;
#ifdef RT_LOOP_STATS
  uint64_t st_cyc[2] = {0, 0}, st_last = 0, st_it[2] = {0, 0}, st_lanes[2] = {0, 0}, st_live = 0;
  // wave-steps, their stepping lanes, wave-steps running the sphere block, leaf lanes, leaf lanes at the
  // first of two sibling leaves (kLeafPair), wave-steps whose leaf lanes are all at such a first leaf
  uint64_t st_step[6] = {0, 0, 0, 0, 0, 0};
  int st_kind = 0;
#endif
  bool mig_ok = false;     // migration gate (wave-uniform) and the time of its next check
  uint64_t mig_next = 0;
  bool have_result = false;  // false: this lane first needs a work item
  uint32_t px_steps = 0;
  int32_t pix = 0;  // (< 2^31: host-checked)
  int s = 0, depth = 0;
  Pcg32 g;
  g.state = 0;
  g.inc = 0;
  g.n = 0;
  uint32_t seg = kItemUnsplit, tc = kNoTarget, st = 0;  // chain render: segment, coupling cursor
  f3 acc = mk(0, 0, 0);
  Record R;
  R.r0 = R.r1 = 0;
  R.n = 0;
  Lane L;
  L.ox = L.oy = L.oz = L.dx = L.dy = L.dz = L.ix = L.iy = L.iz = 0.0f;
  L.a = L.tmax = L.ra = 0.0f;
  L.fast = false;
  L.hit = -1;
  L.cur = 0;

  // chain launches: the heaviest items (the first *n_coop) run on whole waves (coop_items); the lanes'
  // own items start after them
  const int64_t work_offset = kMode == 2 && V.n_coop != nullptr ? (int64_t)*V.n_coop : 0;
  const int64_t total_own = cont ? (int64_t)*V.ch_n_cont
                            : kMode == 2 ? (int64_t)*V.ch_n_items - work_offset
                                         : total - work_offset;

  for (;;) {
    const uint64_t trav = __ballot(mode == kTrav);
    const uint64_t wait = __ballot(mode == kWait);
    if ((trav | wait) == 0) break;
    // shade once shade_batch lanes wait -- or, when fewer lanes are left (the frame's tail), once
    // 3/4 of them do, so a long path is not held back behind its wave's last traversals
    const int live = (int)__popcll(trav | wait);
#if RT_LIVE_PRIO
    // (same box, DESIGN.md §4.1, profiles/r06/ab_live_prio.txt: 3-2-1 at 56-40-24 live lanes against none, the
    // N = 1 chain kernel -1.5 %, the N = 8 / 4 / 2 shares' max rank -6 / -2 / -4 %; sparse waves first: slower)
    if (kMode == 2) {
      if (live >= 56) __builtin_amdgcn_s_setprio(3);
      else if (live >= 40) __builtin_amdgcn_s_setprio(2);
      else if (live >= 24) __builtin_amdgcn_s_setprio(1);
      else __builtin_amdgcn_s_setprio(0);
    }
#endif
    const int batch = min(V.shade_batch, (3 * live + 3) / 4);
    const bool do_trav = trav != 0 && (int)__popcll(wait) < batch;
#ifdef RT_LOOP_STATS
    {  // per wave: iterations, lanes, clocks of traversal vs shading passes
      const uint64_t now = clock64();
      if (st_last) st_cyc[st_kind] += now - st_last;
      st_last = now;
      st_kind = do_trav ? 0 : 1;
      st_it[st_kind]++;
      st_lanes[st_kind] += (uint32_t)__popcll(do_trav ? trav : wait);
      st_live += (uint32_t)live;
    }
#endif
    if (do_trav) {
      // ---------------- traversal steps for every lane still traversing: pass after pass in this
      // inner loop while the wave's shading batch is not full (back through the outer loop's merge
      // after every pass, the compiler shuffled ~90 registers per pass: 6 % of the frame)
      // (in VGPRs: as SGPRs they were re-read from their spill lanes every step)
      uint32_t n9 = (uint32_t)V.n_items9 * 16u, na = (uint32_t)V.n_items9_alloc * 16u;  // (bytes)
      asm volatile("" : "+v"(n9), "+v"(na));
      for (;;) {
        if (mode == kTrav) {
#pragma unroll
          for (int u = 0; u < kSteps; u++) {
#ifdef RT_LOOP_STATS
            {  // per wave-step: stepping lanes, and whether (and for how many lanes) the sphere block runs
              bool at_leaf = false, at_pair = false;
              if (mode == kTrav) {
                const uint32_t hw = __float_as_uint(it_q1(items9, V.n_items9_alloc, L.cur >> 4).w);
                at_leaf = (hw & kLeaf9) != 0u;
                at_pair = at_leaf && (hw & kLeafPair) != 0u;
              }
              const uint64_t stepping = __ballot(mode == kTrav), lm = __ballot(at_leaf), pm = __ballot(at_pair);
              if (stepping) {
                st_step[0]++, st_step[1] += (uint32_t)__popcll(stepping);
                if (lm) st_step[2]++, st_step[3] += (uint32_t)__popcll(lm);
                st_step[4] += (uint32_t)__popcll(pm);
                if (lm && lm == pm) st_step[5]++;
              }
            }
#endif
            if (mode == kTrav) {
              if (kMode == 1) px_steps++;  // work-item cost (the LPT pre-pass)
              if (trav_step_v9(items9, na, n9, L, tmin)) mode = kWait;
            }
          }
        }
        const uint64_t t2 = __ballot(mode == kTrav), w2 = __ballot(mode == kWait);
        const int batch2 = min(V.shade_batch, (3 * (int)__popcll(t2 | w2) + 3) / 4);
        if (t2 == 0ull || (int)__popcll(w2) >= batch2) break;
#ifdef RT_LOOP_STATS
        {
          const uint64_t now = clock64();
          st_cyc[0] += now - st_last;
          st_last = now;
          st_it[0]++;
          st_lanes[0] += (uint32_t)__popcll(t2);
          st_live += (uint32_t)__popcll(t2 | w2);
        }
#endif
      }
      continue;
    }
    if (mode != kWait) continue;
    // migration: the work items are gone (a lane of this wave found none) and few lanes are left
    // and enough of the GPU idles (more than mig_idle waves have become helpers): before that,
    // whole-wave traces would take issue slots from lanes that still make full use of them.  The
    // helper count is read at most every mig_poll ticks per wave (500 us): the device-scope load stalls
    // the wave that needs its value (a load per shading pass from every sparse wave measured 25 % slower
    // lanes; every 20 us, r02-r05a: N = 8 shares 58.7-59.2 ms against 56.0-57.2 at 500 us, N = 1 0.4 %;
    // every 100 us from every dense wave as well: N = 8 +4 ms).
    // (Letting any drained wave migrate once 70-95 % of the waves had finished measured 8 % slower
    // at N = 8: whole-wave traces of dense waves' chains take the helpers from the sparse ones.)
    bool mig_try = false;
    if (kMode == kMigMode && V.mig_live > 0 && live < 64 && live <= V.mig_live) {
      if (!mig_ok) {
        const uint64_t now = wall_clock64();
        if (now >= mig_next) {
          mig_ok = (int32_t)ld_rel(&V.mig[kMigHelpers]) > V.mig_idle;  // (the count only grows)
          mig_next = now + V.mig_poll;
        }
      }
      mig_try = mig_ok;
    }
    // ---------------- shading pass (Camera_ray_color body after hit(), src/raytracing.c:44-75)
    bool need_pixel = !have_result, need_sample = false;
    if (have_result) {
      bool path_done;
      f3 tail = mk(0.0f, 0.0f, 0.0f);
      if (L.hit < 0) {
        tail = ld3(cam.background);
        path_done = true;
      } else {
        // the sphere from its leaf item (LDS): centre in q0, 1/r and the material in q1 -- the same
        // floats as the scene's sphere record, one LDS round trip instead of a global load
        const char *ib = (const char *)items9 + L.hit;
        const float4 c4 = *(const float4 *)ib, h4 = *(const float4 *)(ib + (size_t)V.n_items9_alloc * sizeof(float4));
        const uint32_t mat = __float_as_uint(h4.z);
        const f3 d = mk(L.dx, L.dy, L.dz);
        const f3 p = ray_at(mk(L.ox, L.oy, L.oz), d, L.tmax);
        const f3 outward = scale(sub(p, mk(c4.x, c4.y, c4.z)), h4.y);
        const bool front = dot(d, outward) < 0.0f;
        const f3 normal = front ? outward : neg(outward);
        const FastMat &m = V.mats[mat];
        const f3 nd = scatter(m, normal, front, d, g);
        rec_push(V, R, mat, glane);
        L.ox = p.x, L.oy = p.y, L.oz = p.z;
        L.dx = nd.x, L.dy = nd.y, L.dz = nd.z;
        depth--;
        path_done = depth <= 0;  // the next call would return 0 at depth 0 (src/raytracing.c:40)
      }
      if (path_done) {
        const f3 col = rec_fold(V, R, tail, glane);
        if (kMode == 2 && !(seg & kItemUnsplit) && seg > 0)
          chain_record(V, pix, seg, (uint32_t)s, col, g.n);  // a segment's record
        else
          acc = add(acc, col);
        s++;
        // (the cost pre-pass stops a pixel early once it has spent cost_budget steps: its cost and
        // draws are extrapolated from the samples done, and the pre-pass's latency stays bounded)
        const bool cut = kMode == 1 && px_steps >= V.cost_budget && s < spp;
        if (kMode != 2 && (s == spp || cut)) {  // quantize (src/raytracing.c:127-131)
          if (kMode != 1) write_pixel(out + pix * 3, acc, spp);  // (the pre-pass's image is not used)
          if (kMode == 1) {
            V.cost_out[pix] = cut ? (uint32_t)((uint64_t)px_steps * spp / s) : px_steps;
            V.draw_out[pix] = cut ? (uint32_t)((uint64_t)g.n * spp / s) : g.n;
            if (V.pre_state) V.pre_state[pix] = make_float4(acc.x, acc.y, acc.z, u2f(pre_word(g.n, (uint32_t)s)));
          }
          if (V.px_time) V.px_time[kTimeWords * pix + 1] = (uint32_t)wall_clock64();
          if (kMode == kMigMode && V.mig_live > 0) mig_item_done(V, total_own);
          need_pixel = true;
        } else {
          need_sample = true;
        }
      }
    }
    while (need_pixel || need_sample) {
      if (need_pixel) {  // work stealing among the lanes that need an item right now
        const uint64_t want = __ballot(true);
        const int first = __builtin_ctzll(want);
        int base = 0;
        if (lane == first) base = atomicAdd(V.work_counter, (int)__popcll(want));
        base = __shfl(base, first);
        const int64_t item = (int64_t)base + __popcll(want & ((1ull << lane) - 1));
        if (item >= total_own) {  // no item left: this lane is done
          mode = kExit;
          break;
        }
        acc = mk(0.0f, 0.0f, 0.0f);
        s = 0;
        seg = kItemUnsplit;
        tc = kNoTarget;
        if (kMode == 2 && cont) {  // the true chain on from an exact position (chain_fold_kernel)
          const ChainCont c = V.ch_cont[item];
          pix = (int32_t)c.pix;
          s = (int)c.s;
          acc = mk(c.acc[0], c.acc[1], c.acc[2]);
          st = c.o;  // (applied below, after the seed)
        } else if (kMode == 2) {
          const uint2 it = V.ch_items[item + work_offset];
          pix = (int32_t)it.x;
          seg = it.y;
        } else {
          pix = (int32_t)item;  // (lane launches: low spp / small images, in pixel order)
        }
        {
          const int jj = pix / W, i = pix - jj * W, j = V.row0 + jj * V.row_stride;
          g.seed((uint64_t)(17 + j), (uint64_t)(23 + i));  // src/raytracing.c:94
        }
        if (kMode == 2 && cont) {
          g.skip(st);
        } else if (kMode == 2) {
          if (!(seg & kItemUnsplit)) chain_start(V, (uint32_t)pix, seg, g, tc, st);
          uint32_t s_pre = (uint32_t)s;
          pre_resume(V, pix, seg, g, s_pre, acc);
          s = (int)s_pre;
        }
        need_pixel = false;
        px_steps = 0;
        if (V.px_time && kMode != 2) V.px_time[kTimeWords * pix] = (uint32_t)wall_clock64();
        if (V.px_time && kMode == 2 && !cont) chain_time(V, pix, seg, 0);
      }
      if (kMode == 2 && chain_boundary(V, pix, seg, g.n, (uint32_t)s, acc, tc, st, out, true)) {
        if (kMode == kMigMode && V.mig_live > 0) mig_item_done(V, total_own);
        need_pixel = true;  // this item is finished
        continue;
      }
      if (mig_try && !need_pixel && mig_push(V, (uint32_t)glane % kMigBoxes, pix, seg, (uint32_t)s, acc, g, tc, st)) {
        mode = kExit;  // handed over at this sample boundary
        need_sample = false;
        break;
      }
      // camera ray (src/raytracing.c:96-122)
      const int jj = pix / W, i = pix - jj * W, j = V.row0 + jj * V.row_stride;
      const f3 pixel_pos = add(add(ld3(cam.pixel00), scale(du, (float)i)), scale(dv, (float)j));
      const float px = g.between(-0.5f, 0.5f);
      const float py = g.between(-0.5f, 0.5f);
      f3 o = lf;
      if (dof) {
        float a, b;
        for (;;) {
          a = g.between(-1.0f, 1.0f);
          b = g.between(-1.0f, 1.0f);
          if (a * a + b * b < 1.0f) break;
        }
        o = add(add(lf, scale(ld3(cam.disc_u), a)), scale(ld3(cam.disc_v), b));
      }
      const f3 d = add(add(add(pixel_pos, scale(du, px)), scale(dv, py)), neg(o));
      L.ox = o.x, L.oy = o.y, L.oz = o.z;
      L.dx = d.x, L.dy = d.y, L.dz = d.z;
      depth = max_depth;
      R.n = 0;
      need_sample = false;
      if (depth <= 0) {  // Camera_ray_color returns 0 without tracing (host: chains need depth >= 1)
        acc = add(acc, mk(0.0f, 0.0f, 0.0f));
        s++;
        if (kMode != 2 && s == spp) {
          write_pixel(out + pix * 3, acc, spp);
          if (kMode == kMigMode && V.mig_live > 0) mig_item_done(V, total_own);
          need_pixel = true;
        } else {
          need_sample = true;
        }
      }
    }
    if (mode == kExit) continue;  // (no item: no new ray)
    // set up the traversal of the new ray
    L.ix = 1.0f / L.dx, L.iy = 1.0f / L.dy, L.iz = 1.0f / L.dz;
    L.a = dot(mk(L.dx, L.dy, L.dz), mk(L.dx, L.dy, L.dz));
    L.fast = L.a >= kDivLo && L.a <= kDivHi;
    L.ra = recip_core(L.a);
    L.tmax = __builtin_inff();
    L.hit = -1;
    L.cur = 0u;
    have_result = true;
    mode = V.n_items9 > 0 ? kTrav : kWait;
  }
#ifdef RT_LOOP_STATS
  if (V.loop_stats && __lane_id() == 0) {
    if (st_last) st_cyc[st_kind] += clock64() - st_last;
    unsigned long long *o = V.loop_stats + 8 * kMode;
    atomicAdd(o + 0, (unsigned long long)st_it[0]);
    atomicAdd(o + 1, (unsigned long long)st_lanes[0]);
    atomicAdd(o + 2, (unsigned long long)st_cyc[0]);
    atomicAdd(o + 3, (unsigned long long)st_it[1]);
    atomicAdd(o + 4, (unsigned long long)st_lanes[1]);
    atomicAdd(o + 5, (unsigned long long)st_cyc[1]);
    atomicAdd(o + 6, (unsigned long long)st_live);
    if (kMode == 2)
      for (int q = 0; q < 6; q++) atomicAdd(V.loop_stats + 24 + q, (unsigned long long)st_step[q]);
  }
#endif
  if (kMode == 1 && V.clean_col)  // (the counter: the work-counter line's second half, zeroed with it)
    clean_records(V.clean_col, V.clean_n, (unsigned long long *)(V.work_counter + 16));
  if (kMode == kMigMode && V.mig_live > 0) {
    // (not inlined, so that the whole-wave code does not enlarge the lane loop's register budget; it
    // reads the view from the kernel argument segment -- V is the kernels' first argument -- because
    // taking V's address would copy it to scratch for the whole kernel)
    mig_help<kMode, kLds>(kernarg_view(), out, total_own);
  }
}

// After a chain launch: one lane per split pixel follows the links from segment 0 and sums the
// records in sample order; returns true when the pixel is complete (written to out), else q is its
// continuation item (the exact position its links reach, the colour sum so far).  A segment's records
// are contiguous: eight 16-B loads are in flight before their eight adds, in order.
RT_D bool chain_fold_px(const Book1View &V, uint32_t pix, uint8_t *__restrict__ out, ChainCont &q) {
  const uint32_t spp = (uint32_t)V.S.cam.spp;
  const ChainPx P = V.ch_px[pix];
  uint64_t w = V.ch_seg[P.end0];
  if ((w & kEndEnded) && (w & kEndNoLink)) return true;  // segment 0 wrote the pixel itself
  f3 acc = mk(0.0f, 0.0f, 0.0f);
  uint32_t total = 0, o = 0;
  bool linked = (w & kEndEnded) != 0;  // (segment 0 always ends; not ended would be a bug: start over)
  uint32_t t = 0, c = 0;
  if (linked) {
    const float4 a0 = V.ch_acc0[pix];
    acc = mk(a0.x, a0.y, a0.z);
    total = end_n(w);
    t = end_t(w), c = end_c(w);
    o = c == 0 ? seg_start(P, t) : f2u(V.ch_col[rec_index(P, t, c - 1u)].w);
  }
  while (linked && total < spp) {
    if (t == 0 || t >= P.K) break;  // (never: links point forward)
    w = V.ch_seg[P.end0 + t];
    const uint32_t n = end_n(w);
    const uint32_t m = n > c ? min(n - c, spp - total) : 0u;
    const float4 *rp = V.ch_col + rec_index(P, t, c);
    uint32_t i = 0;
    for (; i + 8u <= m; i += 8u) {
      float4 r[8];
      for (int j = 0; j < 8; j++) r[j] = rp[i + j];
      for (int j = 0; j < 8; j++) acc = add(acc, mk(r[j].x, r[j].y, r[j].z));
      o = f2u(r[7].w);
    }
    for (; i < m; i++) {
      const float4 r = rp[i];
      acc = add(acc, mk(r.x, r.y, r.z));
      o = f2u(r.w);
    }
    total += m;
    if (total >= spp) break;
    if (!(w & kEndEnded) || (w & kEndNoLink)) {
      linked = false;
      break;
    }
    t = end_t(w), c = end_c(w);
  }
  if (total >= spp) {
    write_pixel(out + (size_t)pix * 3, acc, (int)spp);
    return true;
  }
  q.pix = pix, q.o = o, q.s = total, q.pad = 0u;
  q.acc[0] = acc.x, q.acc[1] = acc.y, q.acc[2] = acc.z, q.acc[3] = 0.0f;
  return false;
}

}  // namespace b1
}  // namespace rt
