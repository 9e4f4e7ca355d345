// mgp_api.cpp — the C ABI of libmgpoisson.so (include/mgpoisson.h): level hierarchy, the
// recursive V/F-cycle on one HIP stream, RCCL halo exchange / coarse agglomeration over xGMI,
// and the outer iteration with its fp64 update-RMS.
//
// Reference behaviour reproduced here (thenumbernine/lua-multigrid-poisson):
//   twoGrid recursion         cpu.lua:70-165, cpu-raw.lua:186-237, gpu.lua:296-346
//   fresh / warm coarse guess cpu.lua:138 / cpu-raw.lua:221, gpu.lua:330
//   step / err / run          cpu.lua:196-206, cpu-raw.lua:239-258, gpu.lua:348-373
//   hybrid level hand-off     cpu-gpu.lua:17-52 -> replicated coarse levels after an all-gather
#include "mgp_internal.h"

#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <functional>
#include <optional>
#include <thread>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <map>
#include <vector>

#include <dlfcn.h>

#include "../../include/mgpoisson.h"

using mgp::Geo;

namespace {

thread_local std::string g_create_error;
// Restores the caller's current device on scope exit (the group switches devices per rank).
struct DeviceGuard {
    int dev = -1;
    DeviceGuard() { (void)hipGetDevice(&dev); }
    ~DeviceGuard()
    {
        if (dev >= 0) (void)hipSetDevice(dev);
    }
};

struct LevelPlan {
    int64_t nx, ny, gnz;  // global dims
    int64_t nz, z0;       // local planes / global offset (nz = gnz, z0 = 0 when replicated)
    bool dist;            // slab-decomposed
};

int ilog2(int64_t v)
{
    int l = 0;
    while ((int64_t(1) << l) < v) ++l;
    return l;
}
bool is_pow2(int64_t v) { return v > 0 && (v & (v - 1)) == 0; }

// Host-only hierarchy planner (mgp_plan): coarsen every axis by 2 while all active axes have
// >= 2 cells (cpu.lua recursion down to width 1).  A level stays slab-distributed while its
// planes split evenly with >= 2 per rank, it is not the coarsest and it has more than
// gather_cells cells; from the first replicated level down every rank holds the whole grid.
// MGP_TRANSPORT=rccl (read when a context or group is created): a world-1 3D context takes the slab code path
// on a real one-rank RCCL communicator: ncclGetUniqueId / ncclCommInitRank / ncclCommSplit, the err and norm
// all-reduces, the agglomeration all-gather and the (peerless, empty) grouped halo send/recv all execute.  It is
// how a one-GPU box executes the RCCL transport at all (RCCL refuses two ranks on one device); the results
// equal the plain world-1 run bit for bit (tests/test_gpu_rccl.py).
bool env_rccl1(const mgp_opts& o)
{
    const char* v = std::getenv("MGP_TRANSPORT");
    return o.world == 1 && v && std::strcmp(v, "rccl") == 0;
}

int plan_levels(const mgp_opts& o, std::vector<LevelPlan>& out, std::string& err)
{
    const bool slab1 = env_rccl1(o);
    out.clear();
    if (o.struct_size != (int32_t)sizeof(mgp_opts)) {
        err = "mgp_opts.struct_size mismatch (header/library version skew): fill the struct with this library's "
              "mgp_opts_default";
        return MGP_ERR_ARG;
    }
    if (o.api_version != MGP_API_VERSION) {
        err = "mgp_opts.api_version " + std::to_string(o.api_version) + " != library " + std::to_string(MGP_API_VERSION) +
              " (header/library version skew)";
        return MGP_ERR_ARG;
    }
    if (o.arith != MGP_ARITH_REAL && o.arith != MGP_ARITH_DOUBLE) { err = "unknown arith"; return MGP_ERR_ARG; }
    if (o.dim != 2 && o.dim != 3) { err = "dim must be 2 or 3"; return MGP_ERR_ARG; }
    int64_t nx = o.n[0], ny = o.n[1], nz = o.dim == 3 ? o.n[2] : 1;
    if (!is_pow2(nx) || !is_pow2(ny) || !is_pow2(nz)) { err = "n[] must be powers of two"; return MGP_ERR_ARG; }
    if (nx * ny >= (int64_t(1) << 31)) { err = "nx*ny must be < 2^31"; return MGP_ERR_ARG; }
    if (o.real_bytes != 4 && o.real_bytes != 8) { err = "real_bytes must be 4 or 8"; return MGP_ERR_ARG; }
    if (o.smoother != MGP_JACOBI && o.smoother != MGP_RBGS && o.smoother != MGP_GS_LEX) {
        err = "unknown smoother";
        return MGP_ERR_ARG;
    }
    // cpu.lua's lexicographic sweep is sequential along every axis, so it runs on one rank's whole box only
    if (o.smoother == MGP_GS_LEX && (o.world > 1 || env_rccl1(o))) {
        err = "smoother MGP_GS_LEX (lexicographic, cpu.lua:24-37) is sequential across slabs: world 1 only";
        return MGP_ERR_ARG;
    }

    if (o.cycle != MGP_CYCLE_V && o.cycle != MGP_CYCLE_F) { err = "unknown cycle"; return MGP_ERR_ARG; }
    if (o.prolong != MGP_PROLONG_PC && o.prolong != MGP_PROLONG_LINEAR) { err = "unknown prolong"; return MGP_ERR_ARG; }
    if (o.coarse_init != MGP_COARSE_FRESH && o.coarse_init != MGP_COARSE_WARM) { err = "unknown coarse_init"; return MGP_ERR_ARG; }
    if (o.coarse_bc != MGP_BC_ZERO && o.coarse_bc != MGP_BC_CONSISTENT) { err = "unknown coarse_bc"; return MGP_ERR_ARG; }
    if (o.restriction != MGP_RESTRICT_AVERAGE && o.restriction != MGP_RESTRICT_FULL_WEIGHTING) {
        err = "unknown restriction";
        return MGP_ERR_ARG;
    }
    if (o.nu1 < 0 || o.nu2 < 0 || o.coarse_sweeps < 1) { err = "nu1/nu2 >= 0 and coarse_sweeps >= 1 required"; return MGP_ERR_ARG; }
    if (o.world < 1 || o.rank < 0 || o.rank >= o.world) { err = "need 0 <= rank < world"; return MGP_ERR_ARG; }
    if (o.world > 1) {
        if (o.dim != 3) { err = "domain decomposition is 3D slab-z only"; return MGP_ERR_ARG; }
        if (nz % o.world != 0 || nz / o.world < 2) { err = "n[2] must split into >= 2 planes per rank"; return MGP_ERR_ARG; }
    }
    bool dist = o.world > 1 || (slab1 && o.dim == 3);
    for (;;) {
        LevelPlan p;
        p.nx = nx;
        p.ny = ny;
        p.gnz = nz;
        p.dist = dist;
        p.nz = dist ? nz / o.world : nz;
        p.z0 = dist ? p.nz * o.rank : 0;
        out.push_back(p);
        bool more = nx >= 2 && ny >= 2 && (o.dim == 2 || nz >= 2);
        if (!more || out.size() >= 40) break;
        nx /= 2;
        ny /= 2;
        if (o.dim == 3) nz /= 2;
        bool next_more = nx >= 2 && ny >= 2 && (o.dim == 2 || nz >= 2);
        dist = dist && next_more && nz % o.world == 0 && nz / o.world >= 2 && nx * ny * nz > o.gather_cells;
    }
    return MGP_OK;
}

// the launchers' real kind (mgp_internal.h): float buffers with cpu-raw.lua's double arithmetic, or sizeof(real)
int real_kind(const mgp_opts& o)
{
    return o.real_bytes == 4 && o.arith == MGP_ARITH_DOUBLE ? mgp::kRealF32D : o.real_bytes;
}

double coarse_coef(int coarse_bc, int level)
{
    if (coarse_bc != MGP_BC_CONSISTENT || level <= 0) return 0.0;
    double p = std::ldexp(1.0, level);
    return (p - 1.0) / (p + 1.0);
}

}  // namespace

struct Level {
    LevelPlan p;
    Geo g;
    int64_t alloc;  // reals per buffer, ghost planes included
    char* u = nullptr;
    char* f = nullptr;
    char* t = nullptr;      // second u buffer (Jacobi ping-pong; level 0: keeps psiOld during a cycle)
    bool ghost_ok = true;   // u's ghost planes hold the neighbours' current planes
    bool fghost_ok = true;  // f's ghost planes likewise
    bool fused = false;     // smoothing phases run temporally blocked (k_zs); needs t
    bool blk = false;       // smoothing phases run as 3D-tiled one-launch phases (k_blk); needs t
    bool zpost = false;     // PRE one launch per piece, POST temporally blocked (k_zs); needs t
    bool zero_pending = false;  // u is logically 0: the next red half-sweep reads c->zbuf instead
    bool ghost_zero = false;    // u is 0 everywhere, so ghost planes of any depth are current
    int64_t exchanges = 0;      // halo exchanges of this level so far (mgp_level_info info[7])
    bool early_u = false;       // POST's u halo was exchanged on the side stream after PRE (wait on x_ev1)
    int zc = 0, zc_pre = 0;  // k_zs z-chunks (planes per workgroup) of POST and PRE
};

// Loopback transport (tests): the ranks of a slab decomposition as contexts of one process on
// one GPU, one host thread each; exchanges are device copies ordered by events and a host barrier.
struct mgp_loopback {
    int world = 0;
    std::mutex m;
    std::condition_variable cv;
    int arrived = 0;
    uint64_t gen = 0;
    bool broken = false;
    std::vector<mgp_ctx*> ranks;
    // false after a 120 s wait (a rank failed or stopped calling): the group is then unusable
    bool barrier()
    {
        std::unique_lock<std::mutex> lk(m);
        if (broken) return false;
        const uint64_t g = gen;
        if (++arrived == world) {
            arrived = 0;
            ++gen;
            cv.notify_all();
            return true;
        }
        if (!cv.wait_for(lk, std::chrono::seconds(120), [&] { return gen != g || broken; })) broken = true;
        if (broken) cv.notify_all();
        return !broken;
    }
};

struct mgp_ctx {
    mgp_opts o{};
    int rb = 8;
    // real kind of the per-piece launchers: rb, or mgp::kRealF32D for float buffers with cpu-raw.lua's double
    // arithmetic (mgp_opts.arith = MGP_ARITH_DOUBLE), which runs every level one launch per piece
    int rk = 8;
    int G = 0;  // ghost planes per side (kGhost3D in 3D, 0 in 2D; kGhostZs for distributed 3D)
    bool deep_halo = true;  // smooth_deep on distributed levels below the finest
    bool fresh_sweep = true;        // k_fresh for the first sweep of a lazily zeroed level (MGP_FRESH=0: off)
    bool lazy_zero = true;          // fresh coarse guesses without a memset where a reader can take it (MGP_LAZY_ZERO=0: off)
    bool lazy_zero_fused = true;    // ... on k_zs levels too (their PRE reads none of it; MGP_LAZY_ZERO_FUSED=0: off)
    bool post_black = true;         // the cycle's prolongation corrects the black cells only (MGP_POST_BLACK=0: both)
    bool post1 = false;             // k_post1: prolongation fused into the first post red half-sweep (MGP_POST1=1;
                                    // measured slower: 5 rows of P V per thread cost more VALU and L2 loads
                                    // than the prolongation pass it saves)
    std::vector<Level> lev;
    hipStream_t s = nullptr;
    int device = 0;
    ncclComm_t comm = nullptr;
    // the side stream's own communicator (ncclCommSplit of comm): RCCL runs one communicator's operations in
    // issue order, so the early POST exchange on xs would otherwise hold back every exchange the compute
    // stream issues for the coarse levels until it has finished
    ncclComm_t xcomm = nullptr;
    // host-only dry run (mgp_plan_comm): the cycle's host logic runs, every device and RCCL call is skipped and
    // only the exchange / collective log is kept
    bool dry = false;
    bool nb_comm = false;  // non-blocking communicators (mgp_group_create): every call is polled to completion
    mgp::FusedTuning tu;   // tile settings of the temporally blocked phases (env, snapshot at creation)
    bool resfw = true;     // the full weighting's residual + restriction as one pass (MGP_RESFW=0: two passes)
    bool bres = true;      // the last pre black half-sweep fused with residual + restriction (MGP_BRES=0: apart)
    // whole red/black sweeps of levels below the finest in one pass (MGP_RBSWEEP=1; off by default: at 128^3 11.5 us
    // per sweep against 10.4 for the k_half pair, round 6 — the recomputed edge cells double the VALU of a pass that
    // is latency-bound at that size)
    bool rbsweep = false;
    // PRE of two consecutive small 2D levels in one launch (k_blk2_pre; MGP_BLK2=0: one k_blk launch per level)
    bool blk2 = true;
    bool rccl1 = false;    // world 1 on a one-rank RCCL communicator (MGP_TRANSPORT=rccl, env_rccl1)
    // the multi-rank code path: a communicator (or the loopback transport), collectives, the side stream
    bool multi() const { return o.world > 1 || rccl1; }
    // RCCL API calls of this rank in flight (group_abort waits for them to return before it aborts the
    // communicators) and whether the rank waits on its peers (a halo exchange, collective or the stream
    // synchronisation after one): the group aborts only when a surviving rank is blocked that way
    std::atomic<int> in_nccl{0};
    std::atomic<int> waiting{0};
    mgp_loopback* lb = nullptr;  // loopback transport instead of RCCL (tests)
    hipEvent_t lb_ev = nullptr, lb_ev2 = nullptr;
    // Slab levels: the u halo that a temporally blocked POST reads is final after PRE, so it is exchanged on
    // the side stream xs right after PRE and overlaps the coarse levels (MGP_EARLY_X=0: before POST instead)
    hipStream_t xs = nullptr;
    hipEvent_t x_ev0 = nullptr, x_ev1 = nullptr;
    bool early_x = true;
    char* lb_buf = nullptr;
    double* lb_red = nullptr;
    // psiOld of the last outer iteration (for mgp_metrics), nullptr when not kept
    const char* metrics_old = nullptr;
    double* d_metrics = nullptr;  // 3 * kSumBlocks partials + 3 results
    double* d_rn = nullptr;       // residual-norm partials (+ 2 results), d_rn_cap doubles
    int64_t d_rn_cap = 0;
    char* psi_old = nullptr;  // snapshot buffer (Jacobi path)
    // full-weighting restriction: the residual of the level being restricted (level-0 sized, with ghost planes)
    char* rscratch = nullptr;
    // temporally blocked finest level with err: POST's output buffer, so that psiOld (t) survives the cycle
    // for the reference's metrics (mgp_metrics, psiOld / errorBuf: cpu-raw.lua:148-153, gpu.lua:173-200);
    // rotates with u (MGP_KEEP_PSI_OLD=0: POST writes over psiOld in place and no metrics are kept)
    char* xbuf = nullptr;
    // an all-zero buffer of the largest lazily zeroed level's layout: a fresh coarse guess (cpu.lua:138)
    // costs no memset, the first red half-sweep reads its black neighbours from here
    char* zbuf = nullptr;
    int64_t zbuf_reals = 0;
    char* stage = nullptr;    // lexicographic staging buffer for host set/get (bounded: whole planes in chunks)
    size_t stage_bytes = 0;
    uint64_t* d_stats_h = nullptr;  // mgp_field_stats scratch: kSumBlocks + 1 hashes, then 3 kSumBlocks + 3 doubles
    double* d_part = nullptr;
    std::map<char*, char*> pad_base;  // (MGP_PAD_BYTES) offset pointer -> its allocation
    size_t pad = 0;                   // MGP_PAD_BYTES at creation
    int64_t part_cap = 0;
    double* d_errs = nullptr;
    int errs_cap = 0;
    // one GPU: d_errs is host-pinned mapped memory (h_errs its host side), so mgp_cycles reads the errs after the
    // stream sync without a device-to-host copy (round 6: 25 -> 15 us per call, one-cycle calls 1.079 -> 1.050 ms at
    // 512^3, batched cycles unchanged; MGP_ERRS_HOST=0: device memory and a copy)
    bool errs_host_ok = false, errs_host = false;
    double* h_errs = nullptr;
    // Fused err (red/black): the cycle's first sweep on the finest level runs out of place from u
    // into t, so t keeps psiOld untouched until the last post-sweep, whose two half-sweeps
    // accumulate (psi - psiOld)^2 (cpu.lua:200-203 without the copy and the extra pass).
    bool err_fuse = false;
    bool in_cycle = false;  // a one_cycle() is running (level-0 first sweep goes out of place)
    // set by the owning group when another rank failed: no new exchange / collective is issued, and the
    // communicator (aborted by the group) is not touched again
    const std::atomic<bool>* group_stop = nullptr;
    // a per-process RCCL context whose deadline expired (comm_deadline): its communicators were aborted
    bool comm_dead = false;
    bool stopped() const { return comm_dead || (group_stop && group_stop->load()); }
    const char* stop_msg() const
    {
        return comm_dead ? "communicators aborted after the communication deadline expired (MGP_COMM_TIMEOUT_S)"
                         : "group aborted: another rank failed";
    }
    bool deadline_on() const { return comm_timeout_s > 0.0 && comm && !lb && !nb_comm && !dry; }
    // Deadline of every wait for this rank's streams on a per-process RCCL context (one process per GPU, blocking
    // communicators): MGP_COMM_TIMEOUT_S at creation, default 600 s, 0 = block as before.  An expired wait reports
    // the first exchange / collective whose completion event has not fired, aborts the communicators and fails
    // with MGP_ERR_RCCL (the driver's 8-GPU run must not hang without a record).
    double comm_timeout_s = 0.0;
    struct CommMark {
        hipEvent_t ev = nullptr;
        int op = 0, side = 0, level = 0;
        int64_t seq = -1, bytes = 0;
    };
    std::vector<CommMark> marks;  // ring of completion events of the last calls (kCommMarks)
    int64_t mark_seq = 0;
    static constexpr int kCommMarks = 32;
    // test hook (MGP_TEST_STALL=k, read at creation): the k-th exchange of this context first enqueues a kernel that
    // holds its stream until `stall_flag` is set (or, bounded, 4 x the deadline + 10 s): a peer that never arrives
    int64_t stall_at = 0, exch_seq = 0;
    int* stall_flag = nullptr;    // host-pinned, mapped
    int* stall_flag_d = nullptr;  // its device address
    bool first_done = false;
    bool err_done = false;
    // hipGraph replay of whole cycles (single GPU): one instantiated graph per pointer state of
    // the level buffers (the finest level alternates u/t every cycle), err written to d_errs[*d_slot]
    struct GraphEntry {
        std::vector<char*> pre, post;
        hipGraphExec_t exec = nullptr;
    };
    bool use_graph = false;
    bool use_gs = false;  // grid-stride half-sweeps on large levels (MGP_GS=1; measured slower at 512^3)
    std::vector<GraphEntry> graphs;
    // coarse-level tail (k_tail): cycle_rec(tail_level, ...) as one launch; programs for V and F
    int tail_level = -1;
    std::vector<uint32_t> tail_v, tail_f;
    // hybrid hand-off (cpu-gpu.lua:17-52): the level of size handoff_size goes to a host callback
    int handoff_level = -1;
    mgp_coarse_fn handoff_fn = nullptr;
    void* handoff_user = nullptr;
    std::vector<char> hbuf_u, hbuf_f;
    double* d_err_cur = nullptr;
    double* err_dst = nullptr;  // where this cycle's sum of squares goes
    int* err_ctr = nullptr;     // when set: err_dst[*err_ctr], advanced on the device (mgp_cycles on one GPU)
    int* d_slot = nullptr;      // that device counter
    std::string err;
    // the reference's debugging check (mgp_set_debug): after every phase of a cycle the phase's output is checked
    // for non-finite cells on the device; d_dbg = the first failing check's index into dbg_names (0x7f7f7f7f: none)
    int debug = 0;
    int* d_dbg = nullptr;
    // the last failure was raised after the call's final synchronisation (the debug NaN check): every collective of
    // the call had completed on this rank, so a group's call sequences still match (group_run keeps the group)
    bool fail_after_sync = false;
    std::vector<std::string> dbg_names;
    int dbg_cycle = 0;
    // finest-level kernel timing: event pairs around level-0 launches of each timed kind
    bool timing = false;
    std::vector<hipEvent_t> ev;
    std::vector<std::pair<int, double>> ev_meta;  // (kind, algorithmic bytes) per pair
    size_t ev_used = 0;
    struct CommRec {
        int op, side, level;
        int64_t msgs, bytes;
    };
    static constexpr size_t kCommLogCap = 1 << 16;
    std::vector<CommRec> clog;
    double t_ms[MGP_TIMING_KINDS] = {};
    int64_t t_launch[MGP_TIMING_KINDS] = {};
    double t_bytes[MGP_TIMING_KINDS] = {};
    mgp::LaunchInfo t_info[MGP_TIMING_KINDS] = {};  // the last timed launch of each kernel kind (mgp_timing_kernel)

    int fail(int code, const char* fmt, ...)
    {
        char buf[1024];
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(buf, sizeof buf, fmt, ap);
        va_end(ap);
        err = buf;
        return code;
    }
    char* ui(const Level& L, char* base) const { return base + (size_t)(G * L.g.P) * rb; }
    int64_t ncells_global() const { return lev[0].p.nx * lev[0].p.ny * lev[0].p.gnz; }
    ncclDataType_t nccl_real() const { return rb == 8 ? ncclDouble : ncclFloat; }
};

#define HIP_TRY(c, expr)                                                                         \
    do {                                                                                        \
        if ((c)->dry) break;                                                                    \
        hipError_t e_ = (expr);                                                                 \
        if (e_ != hipSuccess)                                                                   \
            return (c)->fail(MGP_ERR_HIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), \
                             __FILE__, __LINE__);                                               \
    } while (0)

#define NCCL_TRY(c, expr)                                                                           \
    do {                                                                                           \
        if ((c)->dry) break;                                                                       \
        ncclResult_t r_ = (expr);                                                                  \
        if (r_ != ncclSuccess)                                                                     \
            return (c)->fail(MGP_ERR_RCCL, "%s failed: %s (%s:%d)", #expr, ncclGetErrorString(r_), \
                             __FILE__, __LINE__);                                                  \
    } while (0)

#define TRY(expr)                      \
    do {                               \
        int rc_ = (expr);              \
        if (rc_ != MGP_OK) return rc_; \
    } while (0)

namespace {

Geo make_geo(const LevelPlan& p, int dim)
{
    Geo g;
    g.nx = (int)p.nx;
    g.ny = (int)p.ny;
    g.lx = ilog2(p.nx);
    g.ly = ilog2(p.ny);
    g.hw = p.nx >= 2 ? (int)(p.nx / 2) : 1;
    g.lhw = ilog2(g.hw);
    g.nz = dim == 3 ? p.nz : 1;
    g.H = (int64_t)g.hw * g.ny;
    g.P = 2 * g.H;
    g.z0 = dim == 3 ? p.z0 : 0;
    g.gnz = dim == 3 ? p.gnz : 1;
    return g;
}

// ---- halo exchange over RCCL (grouped send/recv to the z-neighbours) ----

// ---- loopback transport (same collective semantics as the RCCL calls below) ----

// The rank waits on its peers while one of these is alive (a transport call, a collective, the stream
// synchronisation or read-back after one): a group aborts a failed rank's peers only when they wait (group_run).
struct WaitScope {
    mgp_ctx* c;
    explicit WaitScope(mgp_ctx* cc) : c(cc) { c->waiting.fetch_add(1); }
    ~WaitScope() { c->waiting.fetch_sub(1); }
};

int lb_fail(mgp_ctx* c) { return c->fail(MGP_ERR_STATE, "loopback group barrier timed out or broken"); }

int lb_exchange(mgp_ctx* c, int l, char* buf, int depth, int colour, hipStream_t st)
{
    WaitScope w(c);
    mgp_loopback* g = c->lb;
    const size_t rb = (size_t)c->rb;
    const Level& L = c->lev[l];
    const size_t bytes = (size_t)(depth * L.g.P) * rb;
    const size_t coff = colour < 0 ? 0 : (size_t)(colour * L.g.H) * rb;  // one colour half per plane
    auto at = [&](char* b, int64_t k) { return b + (size_t)((k + c->G) * L.g.P) * rb + coff; };
    c->lb_buf = buf;
    HIP_TRY(c, hipEventRecord(c->lb_ev, c->s));  // my boundary planes are final here (compute stream)
    if (!g->barrier()) return lb_fail(c);
    const int r = c->o.rank;
    for (int nb : {r - 1, r + 1}) {
        if (nb < 0 || nb >= c->o.world) continue;
        mgp_ctx* o = g->ranks[nb];
        HIP_TRY(c, hipStreamWaitEvent(st, o->lb_ev, 0));
        const char* src = nb < r ? at(o->lb_buf, L.g.nz - depth) : at(o->lb_buf, 0);
        char* dst = nb < r ? at(buf, -depth) : at(buf, L.g.nz);
        if (colour < 0)
            HIP_TRY(c, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, st));
        else
            HIP_TRY(c, hipMemcpy2DAsync(dst, (size_t)L.g.P * rb, src, (size_t)L.g.P * rb, (size_t)L.g.H * rb,
                                        (size_t)depth, hipMemcpyDeviceToDevice, st));
    }
    HIP_TRY(c, hipEventRecord(c->lb_ev2, st));  // my pulls are done here
    if (!g->barrier()) return lb_fail(c);
    for (int nb : {r - 1, r + 1})  // neighbours may overwrite their planes only after my pull
        if (nb >= 0 && nb < c->o.world) HIP_TRY(c, hipStreamWaitEvent(st, g->ranks[nb]->lb_ev2, 0));
    return MGP_OK;
}

// in-place all-gather: rank q's slab is at buf + q * count reals on every rank
int lb_allgather(mgp_ctx* c, char* buf, size_t count)
{
    WaitScope w(c);
    mgp_loopback* g = c->lb;
    const size_t bytes = count * (size_t)c->rb;
    c->lb_buf = buf;
    HIP_TRY(c, hipEventRecord(c->lb_ev, c->s));
    if (!g->barrier()) return lb_fail(c);
    for (int q = 0; q < c->o.world; ++q) {
        if (q == c->o.rank) continue;
        mgp_ctx* o = g->ranks[q];
        HIP_TRY(c, hipStreamWaitEvent(c->s, o->lb_ev, 0));
        HIP_TRY(c, hipMemcpyAsync(buf + q * bytes, o->lb_buf + q * bytes, bytes, hipMemcpyDeviceToDevice, c->s));
    }
    HIP_TRY(c, hipEventRecord(c->lb_ev2, c->s));
    if (!g->barrier()) return lb_fail(c);
    for (int q = 0; q < c->o.world; ++q)
        if (q != c->o.rank) HIP_TRY(c, hipStreamWaitEvent(c->s, g->ranks[q]->lb_ev2, 0));
    return MGP_OK;
}

// in-place sum of n doubles over the ranks, added in rank order
int lb_allreduce(mgp_ctx* c, double* v, int n = 1)
{
    WaitScope w(c);
    mgp_loopback* g = c->lb;
    c->lb_buf = (char*)v;
    HIP_TRY(c, hipEventRecord(c->lb_ev, c->s));
    if (!g->barrier()) return lb_fail(c);
    for (int q = 0; q < c->o.world; ++q) {
        mgp_ctx* o = g->ranks[q];
        if (q != c->o.rank) HIP_TRY(c, hipStreamWaitEvent(c->s, o->lb_ev, 0));
        for (int i = 0; i < n; ++i)
            HIP_TRY(c, hipMemcpyAsync(c->lb_red + i * c->o.world + q, (const double*)o->lb_buf + i, sizeof(double),
                                      hipMemcpyDeviceToDevice, c->s));
    }
    HIP_TRY(c, hipEventRecord(c->lb_ev2, c->s));
    if (!g->barrier()) return lb_fail(c);
    for (int q = 0; q < c->o.world; ++q)
        if (q != c->o.rank) HIP_TRY(c, hipStreamWaitEvent(c->s, g->ranks[q]->lb_ev2, 0));
    for (int i = 0; i < n; ++i) HIP_TRY(c, mgp::launch_sum_partials(c->lb_red + i * c->o.world, c->o.world, v + i, c->s));
    return MGP_OK;
}

// One RCCL call sequence on communicator `comm`: counted in in_nccl for its whole duration (group_abort
// waits for it), refused once the group was stopped, and, on a non-blocking communicator, polled until it
// has left ncclInProgress (returning early when the group is stopped meanwhile).
struct NcclScope {
    mgp_ctx* c;
    explicit NcclScope(mgp_ctx* cc) : c(cc)
    {
        c->in_nccl.fetch_add(1);
        c->waiting.fetch_add(1);
    }
    ~NcclScope()
    {
        c->waiting.fetch_sub(1);
        c->in_nccl.fetch_sub(1);
    }
};

int nccl_done(mgp_ctx* c, ncclComm_t comm, ncclResult_t r, const char* what)
{
    if (r == ncclInProgress || (r == ncclSuccess && c->nb_comm)) {
        for (;;) {
            ncclResult_t st = ncclSuccess;
            r = ncclCommGetAsyncError(comm, &st);
            if (r != ncclSuccess) break;
            if (st != ncclInProgress) {
                r = st;
                break;
            }
            if (c->stopped()) return c->fail(MGP_ERR_STATE, "group aborted during %s", what);
            std::this_thread::yield();
        }
    }
    if (r != ncclSuccess) return c->fail(MGP_ERR_RCCL, "%s: %s", what, ncclGetErrorString(r));
    return MGP_OK;
}

// ---- communication deadline (per-process RCCL contexts) ----

// A completion event after each exchange / collective, in a ring of the last kCommMarks calls: when a wait expires,
// the first of them that has not fired names the call the rank is stuck in.
void comm_mark(mgp_ctx* c, hipStream_t st, int op, int side, int level, int64_t bytes)
{
    if (!c->deadline_on()) return;
    if (c->marks.empty()) {
        c->marks.resize(mgp_ctx::kCommMarks);
        for (auto& m : c->marks)
            if (hipEventCreateWithFlags(&m.ev, hipEventDisableTiming) != hipSuccess) m.ev = nullptr;
    }
    auto& m = c->marks[(size_t)(c->mark_seq % mgp_ctx::kCommMarks)];
    if (!m.ev || hipEventRecord(m.ev, st) != hipSuccess) return;
    m.op = op;
    m.side = side;
    m.level = level;
    m.bytes = bytes;
    m.seq = c->mark_seq++;
}

// The deadline expired while this rank waited for its streams: name what it is stuck in (stderr, so that a bench
// run's tail shows it, and the error text), abort both communicators (their kernels exit) and fail.  The context
// refuses every later exchange / collective; destroy it.  No restart.
int comm_deadline(mgp_ctx* c, double waited)
{
    static const char* ops[] = {"halo exchange", "all-gather", "all-reduce"};
    std::string stuck = "no exchange or collective pending (a kernel of this rank's own stream)";
    for (int64_t k = std::max<int64_t>(0, c->mark_seq - mgp_ctx::kCommMarks); k < c->mark_seq; ++k) {
        const auto& m = c->marks[(size_t)(k % mgp_ctx::kCommMarks)];
        if (m.seq != k || hipEventQuery(m.ev) != hipErrorNotReady) continue;
        char b[200];
        std::snprintf(b, sizeof b, "call #%lld, a %s of level %d on the %s stream (%lld bytes per neighbour)",
                      (long long)k, ops[std::min(2, std::max(0, m.op))], m.level, m.side ? "side" : "compute",
                      (long long)m.bytes);
        stuck = b;
        break;
    }
    std::string recent;
    const size_t n = c->clog.size();
    for (size_t i = n > 4 ? n - 4 : 0; i < n; ++i) {
        const auto& r = c->clog[i];
        char b[96];
        std::snprintf(b, sizeof b, "%s{%s L%d side %d %lld B}", recent.empty() ? "" : ", ",
                      ops[std::min(2, std::max(0, r.op))], r.level, r.side, (long long)r.bytes);
        recent += b;
    }
    c->comm_dead = true;
    if (c->xcomm) (void)ncclCommAbort(c->xcomm);
    if (c->comm) (void)ncclCommAbort(c->comm);
    c->xcomm = c->comm = nullptr;
    if (c->stall_flag) __atomic_store_n(c->stall_flag, 1, __ATOMIC_RELEASE);  // (test hook) release the held stream
    c->fail(MGP_ERR_RCCL,
            "communication deadline: rank %d of %d waited %.1f s (MGP_COMM_TIMEOUT_S=%g) for its streams; stuck in %s; "
            "last issued: %s; communicators aborted",
            c->o.rank, c->o.world, waited, c->comm_timeout_s, stuck.c_str(), recent.c_str());
    std::fprintf(stderr, "mgpoisson: %s\n", c->err.c_str());
    return MGP_ERR_RCCL;
}

// Wait for stream st: hipStreamSynchronize, or, with a deadline, poll the stream and the communicators' async
// errors until it drains or the deadline expires.
int stream_wait(mgp_ctx* c, hipStream_t st)
{
    if (!c->deadline_on()) {
        HIP_TRY(c, hipStreamSynchronize(st));
        return MGP_OK;
    }
    const auto t0 = std::chrono::steady_clock::now();
    for (int spin = 0;; ++spin) {
        const hipError_t q = hipStreamQuery(st);
        if (q == hipSuccess) return MGP_OK;
        if (q != hipErrorNotReady) HIP_TRY(c, q);
        for (ncclComm_t comm : {c->comm, c->xcomm}) {
            ncclResult_t ar = ncclSuccess;
            if (comm && ncclCommGetAsyncError(comm, &ar) == ncclSuccess && ar != ncclSuccess && ar != ncclInProgress)
                return c->fail(MGP_ERR_RCCL, "RCCL async error on rank %d: %s", c->o.rank, ncclGetErrorString(ar));
        }
        const double waited = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (waited > c->comm_timeout_s) return comm_deadline(c, waited);
        if (spin < 4096)
            std::this_thread::yield();
        else
            std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
}

#define NCCL_CALL(c, comm, expr, what)                                                                    \
    do {                                                                                                 \
        if ((c)->dry) break;                                                                             \
        NcclScope scope_(c);                                                                             \
        if ((c)->stopped()) return (c)->fail(MGP_ERR_STATE, "%s", (c)->stop_msg());       \
        TRY(nccl_done((c), (comm), (expr), (what)));                                                     \
    } while (0)

// Exchange `depth` boundary planes of `buf` with each z-neighbour: my first interior planes go to
// rank-1's upper ghosts, my last to rank+1's lower ghosts.  Planes are contiguous in the packed
// layout, so each direction is one ncclSend/ncclRecv pair on that neighbour's xGMI link.
// colour 0 / 1: only that colour's half of each plane (depth pairs of H reals), for readers that never
// look at the other colour (a red/black sweep reads only black cells of its input: the red ones are
// overwritten before they are read), halving the bytes.
// st: the stream the exchange runs on (nullptr: the compute stream; the side stream xs must already wait
// for the compute stream's last write of buf's boundary planes; the loopback transport records that itself)
int timed_begin_on(mgp_ctx* c, hipStream_t st, hipEvent_t* e1);
int timed_end_on(mgp_ctx* c, hipStream_t st, hipEvent_t e1, int kind, double bytes);
void comm_log(mgp_ctx* c, int op, int side, int level, int64_t msgs, int64_t bytes);

int exchange_buf_impl(mgp_ctx* c, Level& L, char* buf, int depth, int colour, hipStream_t st)
{
    if (c->lb) return lb_exchange(c, (int)(&L - c->lev.data()), buf, depth, colour, st);
    const size_t rb = (size_t)c->rb;
    const size_t coff = colour < 0 ? 0 : (size_t)(colour * L.g.H) * rb;
    auto at = [&](int64_t k) { return buf + (size_t)((k + c->G) * L.g.P) * rb + coff; };
    // one message per direction (whole planes) or one per plane (a colour half of each)
    const int msgs = colour < 0 ? 1 : depth;
    const size_t cnt = colour < 0 ? (size_t)(depth * L.g.P) : (size_t)L.g.H;
    ncclComm_t comm = c->xs && st == c->xs && c->xcomm ? c->xcomm : c->comm;
    NcclScope scope(c);
    if (c->stopped()) return c->fail(MGP_ERR_STATE, "%s", c->stop_msg());
    ncclResult_t r = ncclGroupStart();
    for (int i = 0; i < msgs && r == ncclSuccess; ++i) {
        if (c->o.rank > 0) {
            r = ncclSend(at(i), cnt, c->nccl_real(), c->o.rank - 1, comm, st);
            if (r == ncclSuccess) r = ncclRecv(at(i - depth), cnt, c->nccl_real(), c->o.rank - 1, comm, st);
        }
        if (c->o.rank < c->o.world - 1 && r == ncclSuccess) {
            r = ncclSend(at(L.g.nz - depth + i), cnt, c->nccl_real(), c->o.rank + 1, comm, st);
            if (r == ncclSuccess) r = ncclRecv(at(L.g.nz + i), cnt, c->nccl_real(), c->o.rank + 1, comm, st);
        }
    }
    const ncclResult_t e = ncclGroupEnd();  // always closes the group, also after a failed call
    if (r == ncclSuccess) r = e;
    char what[64];
    std::snprintf(what, sizeof what, "halo exchange (level %d)", (int)(&L - c->lev.data()));
    return nccl_done(c, comm, r, what);
}

int exchange_buf(mgp_ctx* c, Level& L, char* buf, int depth = 1, int colour = -1, hipStream_t st = nullptr)
{
    if (!st) st = c->s;
    if (depth > c->G || depth > L.g.nz)
        return c->fail(MGP_ERR_STATE, "internal: exchange depth %d (ghost %d, slab %d)", depth, c->G, (int)L.g.nz);
    if (c->stopped()) return c->fail(MGP_ERR_STATE, "%s", c->stop_msg());
    ++L.exchanges;
    // bytes this rank sends per neighbour: depth planes, or the colour half of each
    const int64_t per_nb = (int64_t)depth * (colour < 0 ? L.g.P : L.g.H) * c->rb;
    const int nbs = (c->o.rank > 0) + (c->o.rank < c->o.world - 1);
    // (side: the xs stream exists and is the one used; a host-only plan without it has s == xs == null)
    comm_log(c, 0, c->xs != nullptr && st == c->xs, (int)(&L - c->lev.data()), colour < 0 ? 1 : depth, per_nb);
    if (c->dry) return MGP_OK;
    hipEvent_t e;
    TRY(timed_begin_on(c, st, &e));
    if (c->stall_at && ++c->exch_seq == c->stall_at && c->stall_flag_d)  // test hook: a peer that never arrives
        HIP_TRY(c, mgp::launch_stall(c->stall_flag_d, 4.0 * c->comm_timeout_s + 10.0, st));
    {
        WaitScope w(c);  // the loopback barrier waits for the peers too
        TRY(exchange_buf_impl(c, L, buf, depth, colour, st));
    }
    comm_mark(c, st, 0, c->xs != nullptr && st == c->xs, (int)(&L - c->lev.data()), per_nb);
    return timed_end_on(c, st, e, MGP_TIMING_EXCHANGE, (double)(per_nb * nbs));
}

int exchange(mgp_ctx* c, Level& L)
{
    if (!L.p.dist || L.ghost_ok) return MGP_OK;
    TRY(exchange_buf(c, L, L.u));
    L.ghost_ok = true;
    return MGP_OK;
}

// ---- finest-level smoother timing ----

void timing_collect(mgp_ctx* c)
{
    for (size_t e = 0; e + 1 < c->ev_used; e += 2) {
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, c->ev[e], c->ev[e + 1]) != hipSuccess) ms = 0.f;
        const auto& m = c->ev_meta[e / 2];
        c->t_ms[m.first] += ms;
        c->t_launch[m.first] += 1;
        c->t_bytes[m.first] += m.second;
    }
    c->ev_used = 0;
}

// An event pair around work on stream st (any level): the exchange and collective kinds
int timed_begin_on(mgp_ctx* c, hipStream_t st, hipEvent_t* e1)
{
    *e1 = nullptr;
    if (!c->timing) return MGP_OK;
    if (c->ev_used + 2 > c->ev.size()) {
        TRY(stream_wait(c, c->s));
        if (c->xs) TRY(stream_wait(c, c->xs));
        timing_collect(c);
    }
    *e1 = c->ev[c->ev_used];
    HIP_TRY(c, hipEventRecord(*e1, st));
    return MGP_OK;
}

int timed_end_on(mgp_ctx* c, hipStream_t st, hipEvent_t e1, int kind, double bytes)
{
    if (!e1) return MGP_OK;
    HIP_TRY(c, hipEventRecord(c->ev[c->ev_used + 1], st));
    c->ev_meta[c->ev_used / 2] = {kind, bytes};
    c->ev_used += 2;
    return MGP_OK;
}

// Level-0 launches on the compute stream: the finest-smoother kinds
int timed_begin(mgp_ctx* c, int l, hipEvent_t* e1)
{
    *e1 = nullptr;
    if (l != 0) return MGP_OK;
    return timed_begin_on(c, c->s, e1);
}

int timed_end(mgp_ctx* c, hipEvent_t e1, int kind, double bytes) { return timed_end_on(c, c->s, e1, kind, bytes); }

// Record of the exchanges and collectives a rank issues (mgp_comm_log): op 0 halo exchange (msgs per
// neighbour and direction, bytes per neighbour), 1 all-gather (bytes of this rank's slab), 2 all-reduce;
// side = issued on the side stream / its communicator.  Bounded: the first kCommLogCap calls after a reset.
void comm_log(mgp_ctx* c, int op, int side, int level, int64_t msgs, int64_t bytes)
{
    if (c->clog.size() < mgp_ctx::kCommLogCap) c->clog.push_back({op, side, level, msgs, bytes});
}

int64_t level_cells(const Level& L) { return L.p.nx * L.p.ny * L.p.nz; }
int64_t level_count(const Level& L) { return L.p.nx * L.p.ny * (L.g.nz); }

// ---- cycle pieces ----

int materialize_zero(mgp_ctx* c, Level& L);

// One half-sweep (colour `color`) reading `other`, writing `dst`; level-0 launches are timed.
// lo / hi > 0: the slab extended by that many ghost planes below / above (deep-halo smoothing).
int half(mgp_ctx* c, int l, int color, char* other, char* dst, const char* old, double h, double cl, int part_off,
         int lo = 0, int hi = 0)
{
    Level& L = c->lev[l];
    Geo g = L.g;
    size_t back = 0;
    if (lo || hi) {
        g.nz += lo + hi;
        g.z0 -= lo;
        back = (size_t)(lo * L.g.P) * c->rb;
    }
    // only the plain finest half-sweep (k_half<T, dim, 1, false>) is timed, so the event total
    // matches that kernel's rocprofv3 row; the err-fused variant reads psiOld as well
    hipEvent_t e;
    TRY(timed_begin(c, old ? -1 : l, &e));
    HIP_TRY(c, mgp::launch_half_sweep(c->rk, c->o.dim, l == 0, color, c->ui(L, other) - back, c->ui(L, L.f) - back,
                                      c->ui(L, dst) - back, old ? c->ui(L, (char*)old) : nullptr, c->d_part + part_off,
                                      g, h, cl, c->use_gs, c->s));
    TRY(timed_end(c, e, MGP_TIMING_HALF_SWEEP, 1.5 * c->rb * (double)level_cells(L)));
    return MGP_OK;
}

// Deep-halo RB-GS on a distributed level below the finest: ONE exchange of D = 2 sweeps + 1 planes
// of u (none when u is a fresh zero) and, once per change of f, of f replaces the exchange before
// every half-sweep.  Half-sweep s computes the slab extended by D - 1 - s ghost planes on every side
// that has a neighbour, redundantly with that neighbour and with the same arithmetic, so the slab's
// own planes are bit-identical to the exchanging schedule and the first ghost plane is current at the
// end (restriction and the level above's prolongation need it).
bool deep_halo_ok(const mgp_ctx* c, const Level& L, int sweeps, bool want_err)
{
    const int l = (int)(&L - c->lev.data());
    const int D = 2 * sweeps + 1;
    return c->deep_halo && l > 0 && L.p.dist && c->o.smoother == MGP_RBGS && !want_err && sweeps >= 1 && D <= c->G &&
           D <= L.g.nz;
}

int smooth_deep(mgp_ctx* c, int l, int sweeps, double h)
{
    Level& L = c->lev[l];
    const double cl = coarse_coef(c->o.coarse_bc, l);
    const int D = 2 * sweeps + 1;
    if (!L.fghost_ok) {  // (the sweeps read f up to D - 1 ghost planes deep)
        TRY(exchange_buf(c, L, L.f, std::min(c->G, (int)L.g.nz)));
        L.fghost_ok = true;
    }
    if (!L.zero_pending && !L.ghost_zero) TRY(exchange_buf(c, L, L.u, D, 1));  // black cells only
    for (int s = 0; s < 2 * sweeps; ++s) {
        const int ext = D - 1 - s;
        const int lo = c->o.rank > 0 ? ext : 0, hi = c->o.rank < c->o.world - 1 ? ext : 0;
        TRY(half(c, l, s & 1, s == 0 && L.zero_pending ? c->zbuf : L.u, L.u, nullptr, h, cl, 0, lo, hi));
        if (s == 0) L.zero_pending = false;
    }
    L.ghost_ok = true;  // the first ghost plane was swept last at extension 1 (black) / 2 (red)
    L.ghost_zero = false;
    return MGP_OK;
}

bool rbsweep_level(const mgp_ctx* c, const Level& L, int l);

// red_done: the first sweep's red half-sweep already ran (k_post1), start at its black half
// black_later: the last sweep's black half-sweep is left to k_bres (black_residual_restrict), which runs it fused
// with the residual and the restriction
int smooth(mgp_ctx* c, int l, int sweeps, double h, bool want_err = false, bool red_done = false,
           bool black_later = false)
{
    Level& L = c->lev[l];
    const double cl = coarse_coef(c->o.coarse_bc, l);
    if (!red_done && deep_halo_ok(c, L, sweeps, want_err)) return smooth_deep(c, l, sweeps, h);
    // a pending zero that no zero-aware path below can read (the tail level swept outside the tail)
    if (L.zero_pending && (c->o.smoother != MGP_RBGS || !c->zbuf || L.alloc > c->zbuf_reals))
        TRY(materialize_zero(c, L));
    for (int sw = 0; sw < sweeps; ++sw) {
        if (c->o.smoother == MGP_GS_LEX) {  // cpu.lua:24-37 in place (a replicated level: validated at creation)
            HIP_TRY(c, mgp::launch_gslex_sweep(c->rk, c->o.dim, c->ui(L, L.u), c->ui(L, L.f), L.g, h, cl, c->s));
            L.ghost_ok = !L.p.dist;
            L.ghost_zero = false;
            continue;
        }
        if (c->o.smoother == MGP_JACOBI) {
            // both colours from the old iterate into t, then swap (no copy back, cf. gpu.lua:292)
            TRY(exchange(c, L));
            TRY(half(c, l, 0, L.u, L.t, nullptr, h, cl, 0));
            TRY(half(c, l, 1, L.u, L.t, nullptr, h, cl, 0));
            std::swap(L.u, L.t);
            L.ghost_ok = !L.p.dist;
            L.ghost_zero = false;
            continue;
        }
        const bool oop = l == 0 && c->in_cycle && c->err_fuse && !c->first_done;  // keep psiOld in t
        const bool last_err = want_err && sw == sweeps - 1;
        if (sw == 0 && L.zero_pending && c->fresh_sweep && !oop && !last_err && !L.p.dist &&
            mgp::fresh_supported(c->rb, L.g)) {
            // the first sweep of a fresh zero guess from f alone (k_fresh: both colours, one pass)
            // with a second sweep to come its red half-sweep replaces the red cells unread: not stored
            HIP_TRY(c, mgp::launch_fresh_sweep(c->rb, c->o.dim, c->ui(L, L.f), c->ui(L, L.u), L.g, h, cl, c->s,
                                               sweeps < 2));
            L.zero_pending = false;
            L.ghost_ok = true;
            L.ghost_zero = false;
            continue;
        }
        if (L.t && rbsweep_level(c, L, l) && !L.zero_pending && !oop && !last_err && !(red_done && sw == 0) &&
            !(black_later && sw == sweeps - 1)) {
            // the whole sweep in one pass into t; its red cells are needed only if no red half-sweep follows
            HIP_TRY(c, mgp::launch_rb_sweep(c->rk, c->o.dim, c->ui(L, L.u), c->ui(L, L.f), c->ui(L, L.t), L.g, h, cl,
                                            sw == sweeps - 1, c->s));
            std::swap(L.u, L.t);
            L.ghost_ok = !L.p.dist;
            L.ghost_zero = false;
            continue;
        }
        const char* old = last_err ? L.t : nullptr;
        const int nb = mgp::half_blocks(c->rk, L.g, c->use_gs);
        char* dst = oop ? L.t : L.u;
        if (!(red_done && sw == 0)) {
            TRY(exchange(c, L));
            TRY(half(c, l, 0, L.zero_pending ? c->zbuf : L.u, dst, old, h, cl, 0));  // red from black
        }
        L.zero_pending = false;
        if (black_later && sw == sweeps - 1 && !oop && !last_err) break;  // (the caller's k_bres runs it)
        if (L.p.dist) {  // black reads the new red planes of dst
            TRY(exchange_buf(c, L, dst));
        }
        TRY(half(c, l, 1, dst, dst, old, h, cl, nb));  // black from red
        if (oop) {
            std::swap(L.u, L.t);  // u = new iterate, t = psiOld (untouched)
            c->first_done = true;
        }
        L.ghost_ok = !L.p.dist;
        L.ghost_zero = false;
        if (last_err) {
            HIP_TRY(c, mgp::launch_sum_partials(c->d_part, 2 * nb, c->err_dst, c->s, c->err_ctr));
            c->err_done = true;
        }
    }
    return MGP_OK;
}

// coarse plane (local to C's storage) and global coarse z of this rank's fine plane 0
Geo coarse_view(const Level& L, const Level& C, int64_t* zc_local)
{
    Geo gc = C.g;
    gc.z0 = L.p.z0 / 2;
    *zc_local = (L.p.dist && !C.p.dist) ? L.p.z0 / 2 : 0;
    return gc;
}

// agglomerate: every rank gets the whole coarse right-hand side R (cf. cpu-gpu.lua:22-32)
int gather_coarse_rhs(mgp_ctx* c, Level& L, Level& C, char* R)
{
    const size_t count = (size_t)((L.g.nz / 2) * C.g.P);
    comm_log(c, 1, 0, (int)(&C - c->lev.data()), 1, (int64_t)(count * c->rb));
    if (c->dry) return MGP_OK;
    hipEvent_t e;
    TRY(timed_begin_on(c, c->s, &e));
    WaitScope w(c);
    if (c->lb)
        TRY(lb_allgather(c, c->ui(C, C.f), count));
    else
        NCCL_CALL(c, c->comm, ncclAllGather(R, c->ui(C, C.f), count, c->nccl_real(), c->comm, c->s), "all-gather");
    comm_mark(c, c->s, 1, 0, (int)(&C - c->lev.data()), (int64_t)(count * c->rb));
    return timed_end_on(c, c->s, e, MGP_TIMING_COLLECTIVE, (double)(count * c->rb * (c->o.world - 1)));
}

// calcResidual + the full-weighting restriction (MGP_RESTRICT_FULL_WEIGHTING): r of the level's own planes
// into the scratch, one ghost plane of r from each z-neighbour on a slab level, then R from r
// the fused residual + full weighting (k_resfw) runs this level (else: r into rscratch, then restrict it)
bool resfw_ok(const mgp_ctx* c, const Level& L)
{
    return c->resfw && mgp::resfw_supported(c->rk, c->o.dim, L.g, c->G, L.p.dist);
}

// The full weighting's level-0 sized residual scratch, when a level the cycle restricts (or, with any_level = false,
// this call) takes the two-pass path: the cycle's levels are checked when the context is created and when its
// coarse engine changes, so that no allocation happens under graph capture.
int ensure_rscratch(mgp_ctx* c, bool cycle_levels, int level = -1)
{
    if (c->rscratch || c->o.restriction != MGP_RESTRICT_FULL_WEIGHTING || c->lev.size() < 2) return MGP_OK;
    bool need = false;
    for (size_t l = 0; l + 1 < c->lev.size(); ++l) {
        const bool used = cycle_levels ? (c->tail_level < 0 || (int)l < c->tail_level) && !c->lev[l].blk
                                       : (int)l == level;
        need = need || (used && !resfw_ok(c, c->lev[l]));
    }
    if (!need) return MGP_OK;
    if (hipMalloc(&c->rscratch, (size_t)c->lev[0].alloc * c->rb) != hipSuccess) {
        c->rscratch = nullptr;
        return c->fail(MGP_ERR_OOM, "hipMalloc failed for the full-weighting residual scratch");
    }
    return MGP_OK;
}

int residual_restrict_fw(mgp_ctx* c, int l, double h)
{
    Level& L = c->lev[l];
    Level& C = c->lev[l + 1];
    TRY(materialize_zero(c, L));
    if (resfw_ok(c, L)) {
        if (L.p.dist) {  // r of the neighbours' first planes: u two planes deep, f one
            TRY(exchange_buf(c, L, L.u, 2));
            L.ghost_ok = true;
            if (!L.fghost_ok) TRY(exchange_buf(c, L, L.f, std::min(c->G, (int)L.g.nz)));
            L.fghost_ok = true;
        }
        int64_t zc = 0;
        const Geo gc = coarse_view(L, C, &zc);
        char* R = c->ui(C, C.f) + (size_t)(zc * C.g.P) * c->rb;
        HIP_TRY(c, mgp::launch_resfw(c->rk, c->o.dim, c->ui(L, L.u), c->ui(L, L.f), R, L.g, gc, h,
                                     coarse_coef(c->o.coarse_bc, l), coarse_coef(c->o.coarse_bc, l + 1), c->G, c->s));
        C.fghost_ok = !C.p.dist;
        if (L.p.dist && !C.p.dist) TRY(gather_coarse_rhs(c, L, C, R));
        return MGP_OK;
    }
    TRY(ensure_rscratch(c, false, l));
    TRY(exchange(c, L));
    HIP_TRY(c, mgp::launch_residual_field_v(c->rk, c->o.dim, c->ui(L, L.u), c->ui(L, L.f), c->ui(L, c->rscratch), L.g,
                                            h, coarse_coef(c->o.coarse_bc, l), c->s));
    if (L.p.dist) TRY(exchange_buf(c, L, c->rscratch, 1));
    int64_t zc = 0;
    const Geo gc = coarse_view(L, C, &zc);
    char* R = c->ui(C, C.f) + (size_t)(zc * C.g.P) * c->rb;
    HIP_TRY(c, mgp::launch_fw_restrict(c->rk, c->o.dim, c->ui(L, c->rscratch), R, L.g, gc,
                                       coarse_coef(c->o.coarse_bc, l + 1), c->s));
    C.fghost_ok = !C.p.dist;
    if (L.p.dist && !C.p.dist) TRY(gather_coarse_rhs(c, L, C, R));
    return MGP_OK;
}

// Pre-smoothing whose last black half-sweep runs fused with the residual and the restriction (k_bres): a replicated
// red/black per-piece level with the average restriction and at least two sweeps (the last one is then a plain red +
// black pair, never the fresh-guess pass).  MGP_BRES=0: the separate half-sweep and k_resrestrict.
bool bres_ok(const mgp_ctx* c, const Level& L)
{
    return c->bres && c->o.smoother == MGP_RBGS && c->o.nu1 >= 2 && c->o.restriction == MGP_RESTRICT_AVERAGE &&
           !L.p.dist && (c->rk == 4 || c->rk == 8) && mgp::bres_supported(c->rk, L.g) && (c->o.dim == 2 || L.g.nz >= 2);
}

// Whole red/black sweeps as one out-of-place pass each (k_rbsweep, u -> t, swapped) on a replicated red/black level
// below the finest (level 0's t is psiOld under the fused err).  MGP_RBSWEEP=0: the k_half pair per sweep.
bool rbsweep_level(const mgp_ctx* c, const Level& L, int l)
{
    return c->rbsweep && c->o.smoother == MGP_RBGS && l > 0 && !L.p.dist && (c->rk == 4 || c->rk == 8) &&
           mgp::bres_supported(c->rk, L.g) && (c->o.dim == 2 || L.g.nz >= 2);
}

int black_residual_restrict(mgp_ctx* c, int l, double h)
{
    Level& L = c->lev[l];
    Level& C = c->lev[l + 1];
    int64_t zc = 0;
    const Geo gc = coarse_view(L, C, &zc);
    char* R = c->ui(C, C.f) + (size_t)(zc * C.g.P) * c->rb;
    HIP_TRY(c, mgp::launch_black_residual_restrict(c->rk, c->o.dim, c->ui(L, L.u), c->ui(L, L.f), R, L.g, gc, h,
                                                   coarse_coef(c->o.coarse_bc, l), c->s));
    L.ghost_ok = true;
    L.ghost_zero = false;
    C.fghost_ok = !C.p.dist;
    return MGP_OK;
}

int residual_restrict(mgp_ctx* c, int l, double h)
{
    if (c->o.restriction == MGP_RESTRICT_FULL_WEIGHTING) return residual_restrict_fw(c, l, h);
    Level& L = c->lev[l];
    Level& C = c->lev[l + 1];
    TRY(materialize_zero(c, L));
    TRY(exchange(c, L));
    int64_t zc = 0;
    const Geo gc = coarse_view(L, C, &zc);
    char* R = c->ui(C, C.f) + (size_t)(zc * C.g.P) * c->rb;
    HIP_TRY(c, mgp::launch_residual_restrict(c->rk, c->o.dim, c->ui(L, L.u), c->ui(L, L.f), R, L.g, gc, h,
                                             coarse_coef(c->o.coarse_bc, l), c->s));
    C.fghost_ok = !C.p.dist;
    if (L.p.dist && !C.p.dist) TRY(gather_coarse_rhs(c, L, C, R));
    return MGP_OK;
}

// black_only: the cycle's correction before a red/black post-smoothing (k_prolong_v skips the red
// cells, which the first post half-sweep replaces without reading)
int prolong_correct(mgp_ctx* c, int l, bool black_only = false)
{
    Level& L = c->lev[l];
    Level& C = c->lev[l + 1];
    const int linear = c->o.prolong == MGP_PROLONG_LINEAR;
    TRY(materialize_zero(c, L));
    TRY(materialize_zero(c, C));
    if (linear && C.p.dist) TRY(exchange(c, C));
    int64_t zc = 0;
    const Geo gc = coarse_view(L, C, &zc);
    char* V = c->ui(C, C.u) + (size_t)(zc * C.g.P) * c->rb;
    HIP_TRY(c, mgp::launch_prolong_correct(c->rk, c->o.dim, linear, c->ui(L, L.u), V, L.g, gc,
                                           coarse_coef(c->o.coarse_bc, l + 1), c->s, black_only));
    L.ghost_ok = !L.p.dist;
    L.ghost_zero = false;
    return MGP_OK;
}

// prolong_correct(l) + the red half of smooth(l, nu2)'s first sweep as one pass (k_post1)
bool post1_ok(const mgp_ctx* c, int l, bool want_err)
{
    const Level& L = c->lev[l];
    const Level& C = c->lev[l + 1];
    int64_t zc = 0;
    return c->post1 && c->o.smoother == MGP_RBGS && c->o.nu2 >= 1 && !(want_err && c->o.nu2 == 1) && !L.p.dist &&
           !C.p.dist && mgp::post1_supported(c->rb, L.g, coarse_view(L, C, &zc));
}

int post_first(mgp_ctx* c, int l, double h)
{
    Level& L = c->lev[l];
    Level& C = c->lev[l + 1];
    TRY(materialize_zero(c, L));
    TRY(materialize_zero(c, C));
    int64_t zc = 0;
    const Geo gc = coarse_view(L, C, &zc);
    char* V = c->ui(C, C.u) + (size_t)(zc * C.g.P) * c->rb;
    HIP_TRY(c, mgp::launch_post_first(c->rb, c->o.dim, c->o.prolong == MGP_PROLONG_LINEAR, c->ui(L, L.u), V,
                                      c->ui(L, L.f), L.g, gc, h, coarse_coef(c->o.coarse_bc, l),
                                      coarse_coef(c->o.coarse_bc, l + 1), c->s));
    L.ghost_ok = true;
    L.ghost_zero = false;
    return MGP_OK;
}

int coarse_solve_at(mgp_ctx* c, int l, double h)
{
    const Level& L = c->lev[l];
    const int64_t cells = L.p.nx * L.p.ny * L.p.gnz;
    return smooth(c, l, cells == 1 ? 1 : c->o.coarse_sweeps, h);
}

// RB-GS levels outside the tail / hand-off / fused levels only need u = 0 as the black input of their
// first red half-sweep (a Gauss-Seidel update never reads the value it replaces, and the black
// half-sweep then reads the new red cells), so their zeroing is deferred to that sweep.  That sweep
// is the first thing the next cycle_rec does on the level only when nu1 >= 1 (the coarsest level's
// solve always sweeps); with nu1 == 0 the residual would read the stale u, so the zero is real then.
bool lazy_zero_ok(const mgp_ctx* c, const Level& L)
{
    const int l = (int)(&L - c->lev.data());
    if (l == c->handoff_level || !c->lazy_zero) return false;
    if (l == c->tail_level) return true;  // run_tail loads it as zeros (any smoother)
    const bool sweeps_first = c->o.nu1 >= 1 || l == (int)c->lev.size() - 1;
    if (L.fused) return c->lazy_zero_fused && c->o.dim == 3 && c->o.nu1 >= 1;  // k_zs PRE loads none of it
    return c->zbuf && sweeps_first && c->o.smoother == MGP_RBGS && L.alloc <= c->zbuf_reals;
}

int zero_level(mgp_ctx* c, Level& L)
{
    if (lazy_zero_ok(c, L)) {
        L.zero_pending = true;
        L.ghost_ok = true;
        L.ghost_zero = true;
        return MGP_OK;
    }
    HIP_TRY(c, hipMemsetAsync(L.u, 0, (size_t)L.alloc * c->rb, c->s));
    L.zero_pending = false;
    L.ghost_ok = true;  // every rank's V is zero, so the ghost planes are current
    L.ghost_zero = true;
    return MGP_OK;
}

// Any reader of u other than the first red half-sweep (the residual, the prolongation of the level
// above, field I/O, a piece called through the ABI) sees a pending lazy zero as a real one.
int materialize_zero(mgp_ctx* c, Level& L)
{
    if (!L.zero_pending) return MGP_OK;
    HIP_TRY(c, hipMemsetAsync(L.u, 0, (size_t)L.alloc * c->rb, c->s));
    L.zero_pending = false;
    L.ghost_ok = true;
    L.ghost_zero = true;
    return MGP_OK;
}

// A level's u, f, t (and the finest level's xbuf) start k * MGP_PAD_BYTES (default 4352 = 4 KiB + 256) into their
// allocations (k = 1, 2, 3, 4).  The arrays are power-of-two sized, so without it equal offsets of u, f, t and xbuf
// share their address bits below 4 KiB, and the phases' concurrent streams of the four arrays meet on the same
// memory channels: 512^3 POST 430 -> 409 us (every offset that is not a multiple of 4 KiB measured alike, 256 B ..
// 64 KiB + 256; multiples of 4 KiB did not help).  MGP_PAD_BYTES=0: no offsets.
size_t pad_bytes()  // (read when a context is created)
{
    const char* e = std::getenv("MGP_PAD_BYTES");
    return e ? (size_t)std::max(0LL, std::atoll(e)) & ~(size_t)255 : (size_t)4352;
}
hipError_t dev_alloc(mgp_ctx* c, char** p, size_t bytes, int k)
{
    const size_t off = (size_t)k * c->pad;
    char* base = nullptr;
    const hipError_t e = hipMalloc(&base, bytes + off);
    if (e != hipSuccess) return e;
    *p = base + off;
    if (off) c->pad_base[*p] = base;
    return hipSuccess;
}
void dev_free(mgp_ctx* c, char* p)
{
    auto it = c->pad_base.find(p);
    (void)hipFree(it == c->pad_base.end() ? p : it->second);
}

double level_h(const mgp_ctx* c, int level) { return std::ldexp(1.0 / (double)c->lev[0].p.nx, level); }

// The black u planes a temporally blocked POST on slab level l reads from its z-neighbours are final once
// PRE has run (the coarse levels never touch them), so they go out on the side stream xs at once and the
// transfer overlaps the coarse levels; fused_post then only waits for x_ev1.  Every rank issues it at the
// same point of the cycle, so the RCCL (and loopback) call order is the same on all ranks.
int early_exchange_post(mgp_ctx* c, int l)
{
    Level& L = c->lev[l];
    if (!c->early_x || !c->xs || !L.p.dist) return MGP_OK;
    // xs waits for PRE on both transports: the ghost planes it writes are read by the compute stream's kernels
    // (the loopback copies additionally wait for the neighbours' events)
    HIP_TRY(c, hipEventRecord(c->x_ev0, c->s));
    HIP_TRY(c, hipStreamWaitEvent(c->xs, c->x_ev0, 0));
    TRY(exchange_buf(c, L, L.u, mgp::kZsHaloPost, 1, c->xs));
    HIP_TRY(c, hipEventRecord(c->x_ev1, c->xs));
    L.early_u = true;
    return MGP_OK;
}

// smooth(l, nu1) + residual_restrict(l) as one temporally blocked pass: u -> t, R -> f of l+1
int fused_pre(mgp_ctx* c, int l, double h)
{
    Level& L = c->lev[l];
    Level& C = c->lev[l + 1];
    if (L.p.dist) {  // the trapezoid reads kZsHaloPre planes of u and f beyond the slab
        // k_zs reads only black cells of its input, and none of a pending fresh zero
        if (!L.zero_pending) TRY(exchange_buf(c, L, L.u, mgp::kZsHaloPre, 1));
        if (!L.fghost_ok) TRY(exchange_buf(c, L, L.f, mgp::kZsHaloPre));
        L.fghost_ok = true;
    }
    int64_t zc = 0;
    const Geo gc = coarse_view(L, C, &zc);
    const bool fw = c->o.restriction == MGP_RESTRICT_FULL_WEIGHTING;
    // the full weighting fused into the phase (fp32 level 0 of one rank's whole box), else smoothing only (both
    // colours stored) and the full weighting after it
    const bool fwf = fw && mgp::fused_fwf_supported(c->rb, c->o.dim, coarse_coef(c->o.coarse_bc, l) == 0.0, L.p.dist, c->tu);
    mgp::FusedArgs a{};
    a.tu = c->tu;
    a.pre = true;
    a.linear = fwf ? 2 : fw;  // PRE: 1 = smoothing only (both colours stored), the full weighting follows
    a.clc = coarse_coef(c->o.coarse_bc, l + 1);  // (the fused full weighting's face weight 3 - c)
    a.src = L.zero_pending ? nullptr : c->ui(L, L.u);  // null: a fresh zero guess (lazy_zero_ok)
    a.f = c->ui(L, L.f);
    a.dst = c->ui(L, L.t);
    a.R = c->ui(C, C.f) + (size_t)(zc * C.g.P) * c->rb;
    a.g = L.g;
    a.gc = gc;
    a.h = h;
    a.cl = coarse_coef(c->o.coarse_bc, l);
    a.zc = L.zc_pre;
    a.ghost = c->G;
    if (l == 0 && c->timing) a.info = &c->t_info[MGP_TIMING_FUSED_PRE];
    hipEvent_t e;
    TRY(timed_begin(c, l, &e));
    HIP_TRY(c, mgp::launch_fused(c->rb, a, c->s));
    // algorithmic bytes (include/mgpoisson.h): read black u and f, write black u and R / 2^dim
    // (full weighting: both colours of u, the restriction runs after the phase)
    const double coarse = std::ldexp(1.0, -c->o.dim);
    TRY(timed_end(c, e, MGP_TIMING_FUSED_PRE, (fw && !fwf ? 2.5 : 2.0 + coarse) * c->rb * (double)level_cells(L)));
    std::swap(L.u, L.t);  // u = smoothed; t = the previous iterate (psiOld on level 0)
    L.zero_pending = false;
    L.ghost_ok = !L.p.dist;
    L.ghost_zero = false;
    if (l == 0 && c->in_cycle) c->first_done = true;
    if (fw && !fwf) return residual_restrict_fw(c, l, h);
    C.fghost_ok = !C.p.dist;
    if (L.p.dist && !C.p.dist) TRY(gather_coarse_rhs(c, L, C, (char*)a.R));  // as residual_restrict
    return MGP_OK;
}

// prolong_correct(l) + smooth(l, nu2) as one temporally blocked pass: u + P V -> t (err vs t)
int fused_post(mgp_ctx* c, int l, double h, bool want_err)
{
    Level& L = c->lev[l];
    Level& C = c->lev[l + 1];
    if (L.p.dist) {  // kZsHaloPost planes of u and f, kZsHaloCoarse coarse planes of V
        if (L.early_u) {  // exchanged on xs after PRE (early_exchange_post)
            HIP_TRY(c, hipStreamWaitEvent(c->s, c->x_ev1, 0));
            L.early_u = false;
        } else {
            TRY(exchange_buf(c, L, L.u, mgp::kZsHaloPost, 1));
        }
        if (!L.fghost_ok) TRY(exchange_buf(c, L, L.f, mgp::kZsHaloPost));
        L.fghost_ok = true;
        if (C.p.dist) TRY(exchange_buf(c, C, C.u, mgp::kZsHaloCoarse));
    }
    int64_t zc = 0;
    const Geo gc = coarse_view(L, C, &zc);
    mgp::FusedArgs a{};
    a.tu = c->tu;
    a.pre = false;
    a.linear = c->o.prolong == MGP_PROLONG_LINEAR;
    a.src = c->ui(L, L.u);
    a.f = c->ui(L, L.f);
    // with err on level 0: t holds psiOld; the output goes to xbuf when psiOld is kept, else over t
    const bool keep = want_err && l == 0 && c->xbuf;
    a.dst = c->ui(L, keep ? c->xbuf : L.t);
    a.old = want_err ? c->ui(L, L.t) : nullptr;
    a.V = c->ui(C, C.u) + (size_t)(zc * C.g.P) * c->rb;
    a.partials = want_err ? c->d_part : nullptr;
    if (c->tu.stamp_r) a.R = c->ui(C, C.f);  // (ZS_STAMP timing builds: POST's stamps into level l+1's f)
    a.g = L.g;
    a.gc = gc;
    a.h = h;
    a.cl = coarse_coef(c->o.coarse_bc, l);
    a.clc = coarse_coef(c->o.coarse_bc, l + 1);
    a.zc = L.zc;
    a.ghost = c->G;
    if (l == 0 && c->timing) a.info = &c->t_info[MGP_TIMING_FUSED_POST];
    hipEvent_t e;
    TRY(timed_begin(c, l, &e));
    HIP_TRY(c, mgp::launch_fused(c->rb, a, c->s));
    // read black u, V / 2^dim, f (and psiOld with err), write u
    TRY(timed_end(c, e, MGP_TIMING_FUSED_POST,
                  (2.5 + std::ldexp(1.0, -c->o.dim) + (want_err ? 1.0 : 0.0)) * c->rb * (double)level_cells(L)));
    if (keep)
        std::swap(L.u, c->xbuf);  // u = new iterate, t = psiOld (kept), xbuf = the smoothed PRE output (scratch)
    else
        std::swap(L.u, L.t);
    L.ghost_ok = !L.p.dist;
    L.ghost_zero = false;
    if (want_err) {
        HIP_TRY(c, mgp::launch_sum_partials(c->d_part,
                                            mgp::fused_blocks(c->rb, L.g, L.zc, coarse_coef(c->o.coarse_bc, l) == 0.0, c->tu),
                                            c->err_dst, c->s, c->err_ctr));
        c->err_done = true;
    }
    return MGP_OK;
}

// smooth(l, nu1) + residual_restrict(l) of a small replicated level as one 3D-tiled launch:
// u -> t, R -> f of l+1 (a pending fresh zero is read as such, no memset)
int block_pre(mgp_ctx* c, int l, double h)
{
    Level& L = c->lev[l];
    Level& C = c->lev[l + 1];
    int64_t zc = 0;
    mgp::BlockArgs a{};
    a.pre = true;
    a.ns = c->o.nu1;
    a.src = L.zero_pending ? nullptr : c->ui(L, L.u);
    a.f = c->ui(L, L.f);
    a.dst = c->ui(L, L.t);
    a.g = L.g;
    a.gc = coarse_view(L, C, &zc);
    a.R = c->ui(C, C.f) + (size_t)(zc * C.g.P) * c->rb;
    a.h = h;
    a.cl = coarse_coef(c->o.coarse_bc, l);
    a.linear = c->o.restriction == MGP_RESTRICT_FULL_WEIGHTING;  // PRE: the restriction
    a.clc = coarse_coef(c->o.coarse_bc, l + 1);
    HIP_TRY(c, mgp::launch_block(c->rb, c->o.dim, a, c->s));
    L.zero_pending = false;
    std::swap(L.u, L.t);
    L.ghost_ok = true;
    L.ghost_zero = false;
    C.fghost_ok = true;
    return MGP_OK;
}

// block_pre(l), the fresh guess of l + 1 and block_pre(l + 1) as one launch (k_blk2_pre): two consecutive k_blk 2D
// levels of a V-cycle (average restriction, fp32; the tile divides level l + 1).  The state afterwards is the same as
// after the three steps: u of both levels smoothed (black cells), f of l + 1 and l + 2 restricted.
// block_post(l + 1) and block_post(l) likewise (k_blk2_post).  Both pair level l with l + 1 in the V-cycle part of a
// cycle (cycle_rec with fcycle false).
bool pair2_ok(const mgp_ctx* c, int l, double h, bool fcycle, int ns)
{
    const int last = (int)c->lev.size() - 1;
    if (!c->blk2 || fcycle || l + 2 > last || (c->rk != 4 && c->rk != 8) || c->o.dim != 2 || c->o.smoother != MGP_RBGS)
        return false;
    if (l + 1 == c->tail_level || l + 1 == c->handoff_level || h != level_h(c, l)) return false;
    const Level &L = c->lev[l], &C = c->lev[l + 1], &D = c->lev[l + 2];
    if (!L.blk || !C.blk || L.fused || C.fused || L.p.dist || C.p.dist || D.p.dist) return false;
    return mgp::block2_supported(c->rb, c->o.dim, ns, L.g, C.g, D.g);
}
bool pre2_ok(const mgp_ctx* c, int l, double h, bool fcycle)
{
    return c->o.restriction != MGP_RESTRICT_FULL_WEIGHTING && pair2_ok(c, l, h, fcycle, c->o.nu1);
}
bool post2_ok(const mgp_ctx* c, int l, double h, bool fcycle) { return pair2_ok(c, l, h, fcycle, c->o.nu2); }

int block_pre2(mgp_ctx* c, int l, double h)
{
    Level& L = c->lev[l];
    Level& C = c->lev[l + 1];
    Level& D = c->lev[l + 2];
    int64_t zc = 0, zc2 = 0;
    mgp::Block2Args a{};
    a.pre = true;
    a.ns = c->o.nu1;
    a.src = L.zero_pending ? nullptr : c->ui(L, L.u);
    a.f = c->ui(L, L.f);
    a.dst = c->ui(L, L.t);
    a.g = L.g;
    a.g1 = coarse_view(L, C, &zc);
    a.f1 = c->ui(C, C.f) + (size_t)(zc * C.g.P) * c->rb;
    // level l + 1's guess: cycle_rec's fresh zero (cpu.lua:138), or the warm one unless a zero is pending
    const bool fresh1 = c->o.coarse_init == MGP_COARSE_FRESH || C.zero_pending;
    a.src1 = fresh1 ? nullptr : c->ui(C, C.u);
    a.dst1 = c->ui(C, C.t);
    a.g2 = coarse_view(C, D, &zc2);
    a.R = c->ui(D, D.f) + (size_t)(zc2 * D.g.P) * c->rb;
    a.h = h;
    a.cl = coarse_coef(c->o.coarse_bc, l);
    a.cl1 = coarse_coef(c->o.coarse_bc, l + 1);
    HIP_TRY(c, mgp::launch_block2(c->rb, c->o.dim, a, c->s));
    L.zero_pending = false;
    std::swap(L.u, L.t);
    L.ghost_ok = true;
    L.ghost_zero = false;
    C.fghost_ok = true;
    C.zero_pending = false;
    std::swap(C.u, C.t);
    C.ghost_ok = true;
    C.ghost_zero = false;
    D.fghost_ok = true;
    return MGP_OK;
}

int block_post2(mgp_ctx* c, int l, double h)
{
    Level& L = c->lev[l];
    Level& C = c->lev[l + 1];
    Level& D = c->lev[l + 2];
    TRY(materialize_zero(c, L));
    TRY(materialize_zero(c, C));
    TRY(materialize_zero(c, D));
    mgp::Block2Args a{};
    a.pre = false;
    a.linear = c->o.prolong == MGP_PROLONG_LINEAR;
    a.ns = c->o.nu2;
    a.src = c->ui(L, L.u);
    a.f = c->ui(L, L.f);
    a.dst = c->ui(L, L.t);
    a.src1 = c->ui(C, C.u);
    a.f1 = c->ui(C, C.f);
    a.dst1 = c->ui(C, C.t);
    a.V2 = c->ui(D, D.u);
    a.g = L.g;
    a.g1 = C.g;
    a.g2 = D.g;
    a.h = h;
    a.cl = coarse_coef(c->o.coarse_bc, l);
    a.cl1 = coarse_coef(c->o.coarse_bc, l + 1);
    a.cl2 = coarse_coef(c->o.coarse_bc, l + 2);
    HIP_TRY(c, mgp::launch_block2(c->rb, c->o.dim, a, c->s));
    std::swap(C.u, C.t);
    C.ghost_ok = true;
    C.ghost_zero = false;
    std::swap(L.u, L.t);
    L.ghost_ok = true;
    L.ghost_zero = false;
    return MGP_OK;
}

// prolong_correct(l) + smooth(l, nu2) of a small replicated level as one 3D-tiled launch: u + P V -> t
int block_post(mgp_ctx* c, int l, double h)
{
    Level& L = c->lev[l];
    Level& C = c->lev[l + 1];
    TRY(materialize_zero(c, L));
    TRY(materialize_zero(c, C));
    int64_t zc = 0;
    mgp::BlockArgs a{};
    a.pre = false;
    a.linear = c->o.prolong == MGP_PROLONG_LINEAR;
    a.ns = c->o.nu2;
    a.src = c->ui(L, L.u);
    a.f = c->ui(L, L.f);
    a.dst = c->ui(L, L.t);
    a.g = L.g;
    a.gc = coarse_view(L, C, &zc);
    a.V = c->ui(C, C.u) + (size_t)(zc * C.g.P) * c->rb;
    a.h = h;
    a.cl = coarse_coef(c->o.coarse_bc, l);
    a.clc = coarse_coef(c->o.coarse_bc, l + 1);
    HIP_TRY(c, mgp::launch_block(c->rb, c->o.dim, a, c->s));
    std::swap(L.u, L.t);
    L.ghost_ok = true;
    L.ghost_zero = false;
    return MGP_OK;
}

// The ops of cycle_rec(l, fcycle) for levels >= T, recorded for k_tail (levels relative to T).
void tail_gen(const mgp_ctx* c, int T, int l, bool fcycle, std::vector<uint32_t>& ops)
{
    auto emit = [&](int op, int lv, int arg) {
        ops.push_back((uint32_t)op | ((uint32_t)(lv - T) << 4) | ((uint32_t)arg << 8));
    };
    const int last = (int)c->lev.size() - 1;
    if (l == last) {
        const Level& L = c->lev[l];
        const int64_t cells = L.p.nx * L.p.ny * L.p.gnz;
        emit(mgp::TAIL_SMOOTH, l, cells == 1 ? 1 : c->o.coarse_sweeps);
        return;
    }
    emit(mgp::TAIL_SMOOTH, l, c->o.nu1);
    emit(mgp::TAIL_RR, l, 0);
    if (c->o.coarse_init == MGP_COARSE_FRESH) emit(mgp::TAIL_ZERO, l + 1, 0);
    if (fcycle) tail_gen(c, T, l + 1, true, ops);
    tail_gen(c, T, l + 1, false, ops);
    emit(mgp::TAIL_PROLONG, l, 0);
    emit(mgp::TAIL_SMOOTH, l, c->o.nu2);
}

// First level (>= 1, replicated, <= MGP_TAIL_CELLS cells) whose sub-hierarchy fits one
// workgroup's LDS and the op budget; -1 = no tail (MGP_TAIL=0 disables it).
// Make level T (>= 1, replicated) the first level of the coarse tail if its sub-hierarchy fits
// one workgroup's LDS and the op budget.
bool try_tail(mgp_ctx* c, int T)
{
    const int last = (int)c->lev.size() - 1;
    if (T < 1 || T > last || c->lev[T].p.dist) return false;
    if (c->rk == mgp::kRealF32D) return false;  // the tail evaluates in the real type
    if (c->o.smoother == MGP_GS_LEX) return false;  // the tail runs Jacobi and red/black sweeps only
    const int nlev = last - T + 1;
    if (nlev > mgp::kTailMaxLevels) return false;
    std::vector<Geo> g;
    for (int l = T; l <= last; ++l) g.push_back(c->lev[l].g);
    if (mgp::tail_lds_bytes(c->rb, c->o.dim, c->o.smoother == MGP_JACOBI, g.data(), nlev) > mgp::kTailMaxLds)
        return false;
    std::vector<uint32_t> pv, pf;
    tail_gen(c, T, T, false, pv);
    tail_gen(c, T, T, true, pf);
    if ((int)pv.size() > mgp::kTailMaxOps || (int)pf.size() > mgp::kTailMaxOps) return false;
    c->tail_level = T;
    c->tail_v = pv;
    c->tail_f = pf;
    return true;
}

// Default: the first level with <= MGP_TAIL_CELLS (4096) cells that fits (MGP_TAIL=0: none).
void plan_tail(mgp_ctx* c)
{
    c->tail_level = -1;
    const char* v = std::getenv("MGP_TAIL");
    if (v && std::atoi(v) == 0) return;
    const char* vc = std::getenv("MGP_TAIL_CELLS");
    const int64_t max_cells = vc ? std::atoll(vc) : 4096;
    for (int T = 1; T < (int)c->lev.size(); ++T) {
        const Level& L = c->lev[T];
        if (L.p.nx * L.p.ny * L.p.gnz <= max_cells && try_tail(c, T)) return;
    }
}

void drop_graphs(mgp_ctx* c)
{
    for (auto& g : c->graphs) (void)hipGraphExecDestroy(g.exec);
    c->graphs.clear();
}

// cpu-gpu.lua:17-52: level l's u and f to the host, the callback's coarse cycle, and back
int run_handoff(mgp_ctx* c, int l, double h)
{
    Level& L = c->lev[l];
    const int64_t n = level_count(L);
    c->hbuf_u.resize((size_t)n * c->rb);
    c->hbuf_f.resize((size_t)n * c->rb);
    TRY(mgp_get_field(c, l, MGP_FIELD_U, c->hbuf_u.data(), n, MGP_MEM_HOST));
    TRY(mgp_get_field(c, l, MGP_FIELD_F, c->hbuf_f.data(), n, MGP_MEM_HOST));
    const int rc = c->handoff_fn(c->handoff_user, h, c->hbuf_u.data(), c->hbuf_f.data(), L.p.nx);
    if (rc != 0) return c->fail(MGP_ERR_STATE, "coarse hand-off callback returned %d", rc);
    TRY(mgp_set_field(c, l, MGP_FIELD_U, c->hbuf_u.data(), n, MGP_MEM_HOST));
    TRY(mgp_set_field(c, l, MGP_FIELD_F, c->hbuf_f.data(), n, MGP_MEM_HOST));
    L.ghost_ok = !L.p.dist;
    L.ghost_zero = false;
    return MGP_OK;
}

int run_tail(mgp_ctx* c, bool fcycle)
{
    mgp::TailSpec t{};
    const int T = c->tail_level, last = (int)c->lev.size() - 1;
    t.nlev = last - T + 1;
    t.jacobi = c->o.smoother == MGP_JACOBI;
    t.linear = c->o.prolong == MGP_PROLONG_LINEAR;
    for (int i = 0; i < t.nlev; ++i) {
        Level& L = c->lev[T + i];
        t.u[i] = c->ui(L, L.u);
        t.f[i] = c->ui(L, L.f);
        t.g[i] = L.g;
        t.h[i] = level_h(c, T + i);
        t.cl[i] = coarse_coef(c->o.coarse_bc, T + i);
        L.ghost_ok = true;
        L.ghost_zero = false;
    }
    t.zero_first = c->lev[T].zero_pending;
    t.fw = c->o.restriction == MGP_RESTRICT_FULL_WEIGHTING;
    c->lev[T].zero_pending = false;
    const std::vector<uint32_t>& p = fcycle ? c->tail_f : c->tail_v;
    t.nops = (int)p.size();
    std::copy(p.begin(), p.end(), t.ops);
    HIP_TRY(c, mgp::launch_tail(c->rb, c->o.dim, t, c->s));
    return MGP_OK;
}

// ---- roctx ranges (SURVEY.md §5 tracing): MGP_ROCTX=1 names the cycle and every level's phases on the host
// timeline of rocprofv3 --marker-trace.  The roctx library is opened at run time (no link dependency); graph
// replay is off while ranges are on, so every cycle enqueues (and names) its launches.
struct Roctx {
    int (*push)(const char*) = nullptr;
    int (*pop)() = nullptr;
    Roctx()
    {
        const char* v = std::getenv("MGP_ROCTX");
        if (!(v && std::atoi(v))) return;
        void* h = dlopen("librocprofiler-sdk-roctx.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen("libroctx64.so.4", RTLD_NOW | RTLD_LOCAL);
        if (!h) return;
        push = reinterpret_cast<int (*)(const char*)>(dlsym(h, "roctxRangePushA"));
        pop = reinterpret_cast<int (*)()>(dlsym(h, "roctxRangePop"));
        if (!push || !pop) push = nullptr, pop = nullptr;
    }
};
const Roctx& roctx()
{
    static const Roctx r;
    return r;
}
bool roctx_on() { return roctx().push != nullptr; }
struct Range {
    bool on;
    Range(const char* fmt, int l) : on(roctx_on())
    {
        if (!on) return;
        char b[64];
        std::snprintf(b, sizeof(b), fmt, l);
        roctx().push(b);
    }
    ~Range()
    {
        if (on) roctx().pop();
    }
};

// mgp_set_debug: check level l's `buf` (u or f) for non-finite cells after the phase `what` (cpu-raw.lua:126-140
// show + "found a nan", called after every smoother sweep / residual / restriction / prolongation there)
int debug_check(mgp_ctx* c, int l, const char* what, bool f_field = false)
{
    if (!c->debug || c->dry || !c->d_dbg) return MGP_OK;
    Level& L = c->lev[l];
    if (!f_field && L.zero_pending) return MGP_OK;  // a pending fresh zero
    char name[160];
    std::snprintf(name, sizeof name, "cycle %d, level %d (%lld x %lld x %lld), %s", c->dbg_cycle, l, (long long)L.p.nx,
                  (long long)L.p.ny, (long long)(c->o.dim == 3 ? L.g.nz : 1), what);
    const int id = (int)c->dbg_names.size();
    c->dbg_names.push_back(name);
    HIP_TRY(c, mgp::launch_nonfinite_check(c->rb, c->ui(L, f_field ? L.f : L.u), L.g.P * L.g.nz, id, c->d_dbg, c->s));
    return MGP_OK;
}

// pre_done: the level above ran this level's pre-smoothing and restriction in its launch (block_pre2); post_skip: the
// level above runs this level's prolongation and post-smoothing in its launch (block_post2)
int cycle_rec(mgp_ctx* c, int l, double h, bool fcycle, bool pre_done = false, bool post_skip = false)
{
    const int last = (int)c->lev.size() - 1;
    if (l == c->handoff_level && c->handoff_fn) {
        Range r("L%d hand-off", l);
        return run_handoff(c, l, h);
    }
    if (l == c->tail_level && h == level_h(c, l)) {
        Range r("L%d+ coarse tail", l);
        TRY(run_tail(c, fcycle));
        return debug_check(c, l, "the coarse tail (V = its cycle)");
    }
    if (l == last) {
        Range r("L%d coarse solve", l);
        TRY(coarse_solve_at(c, l, h));
        return debug_check(c, l, "the coarse solve");
    }
    const bool fused = c->lev[l].fused && h == level_h(c, l);
    const bool blk = !fused && c->lev[l].blk && h == level_h(c, l);
    const bool zpost = c->lev[l].zpost && h == level_h(c, l);
    std::optional<Range> pre_range(std::in_place, "L%d pre-smooth + restrict", l);
    const bool pre2 = !pre_done && blk && pre2_ok(c, l, h, fcycle);
    if (pre_done) {
    } else if (fused) {
        TRY(fused_pre(c, l, h));
        TRY(early_exchange_post(c, l));
    } else if (pre2) {
        TRY(block_pre2(c, l, h));
    } else if (blk) {
        TRY(block_pre(c, l, h));
    } else if (bres_ok(c, c->lev[l])) {
        TRY(smooth(c, l, c->o.nu1, h, false, false, true));
        TRY(black_residual_restrict(c, l, h));
    } else {
        TRY(smooth(c, l, c->o.nu1, h));
        TRY(residual_restrict(c, l, h));
    }
    TRY(debug_check(c, l, "pre-smoothing (u)"));
    TRY(debug_check(c, l + 1, pre2 ? "the restriction and its pre-smoothing (block_pre2)"
                                   : "the restriction (R = f of the coarse level)", true));
    // (block_pre2 already smoothed level l + 1 from its fresh guess)
    if (c->o.coarse_init == MGP_COARSE_FRESH && !pre2) TRY(zero_level(c, c->lev[l + 1]));
    pre_range.reset();
    const bool want_err = l == 0 && c->in_cycle && c->err_fuse;
    const bool post2 = !post_skip && blk && !want_err && post2_ok(c, l, h, fcycle);  // (pairs like pre2)
    if (fcycle) TRY(cycle_rec(c, l + 1, 2 * h, true));
    TRY(cycle_rec(c, l + 1, 2 * h, false, pre2, post2));
    if (post_skip) return MGP_OK;  // (block_post2 of the level above)
    Range post_range("L%d prolong + post-smooth", l);
    if (fused || zpost) {
        TRY(fused_post(c, l, h, want_err));
    } else if (post2) {
        TRY(block_post2(c, l, h));
        TRY(debug_check(c, l + 1, "the prolongation + correction and post-smoothing (u, block_post2)"));
    } else if (blk && !want_err) {
        TRY(block_post(c, l, h));
    } else if (post1_ok(c, l, want_err)) {
        TRY(post_first(c, l, h));
        TRY(smooth(c, l, c->o.nu2, h, want_err, true));
    } else {
        TRY(prolong_correct(c, l, c->post_black && c->o.smoother == MGP_RBGS && c->o.nu2 >= 1));
        TRY(smooth(c, l, c->o.nu2, h, want_err));
    }
    return debug_check(c, l, "the prolongation + correction and post-smoothing (u)");
}

// Where the last outer iteration's psiOld lives: the level-0 t buffer with the fused err (the
// first sweep ran out of place), the snapshot otherwise; lost when the temporally blocked phase
// overwrote it, absent without err_mode.
void update_metrics_old(mgp_ctx* c)
{
    const Level& L0 = c->lev[0];
    c->metrics_old = nullptr;
    if (!c->o.err_mode) return;
    if (!c->err_fuse)
        c->metrics_old = c->psi_old;
    else if (!L0.fused || c->xbuf)
        c->metrics_old = c->ui(L0, L0.t);
}

// One outer iteration; err (sum of squares) goes to *dst.
int one_cycle(mgp_ctx* c, double* dst)
{
    Level& L = c->lev[0];
    const size_t bytes = (size_t)(L.g.P * L.g.nz) * c->rb;
    const bool fuse = c->o.err_mode && c->err_fuse;
    c->err_dst = dst;
    c->err_done = false;
    c->first_done = false;
    if (c->o.err_mode && !fuse)
        HIP_TRY(c, hipMemcpyAsync(c->psi_old, c->ui(L, L.u), bytes, hipMemcpyDeviceToDevice, c->s));
    const double h = 1.0 / (double)L.p.nx;  // cpu.lua:197-198
    c->in_cycle = true;
    int rc;
    {
        Range r(c->o.cycle == MGP_CYCLE_F ? "F-cycle%.0d" : "V-cycle%.0d", 0);
        rc = cycle_rec(c, 0, h, c->o.cycle == MGP_CYCLE_F);
    }
    c->in_cycle = false;
    TRY(rc);
    if (fuse && !c->err_done) return c->fail(MGP_ERR_STATE, "internal: fused err launch did not run");
    if (c->o.err_mode && !fuse) {
        Level& L0 = c->lev[0];
        HIP_TRY(c, mgp::launch_sqdiff_sum(c->rk, c->ui(L0, L0.u), c->psi_old, L0.g.P * L0.g.nz, c->d_part, dst, c->s,
                                          c->err_ctr));
    }
    if (c->o.err_mode && c->multi()) {
        comm_log(c, 2, 0, 0, 1, (int64_t)sizeof(double));
        if (c->dry) return MGP_OK;
        hipEvent_t e;
        TRY(timed_begin_on(c, c->s, &e));
        WaitScope w(c);
        if (c->lb)
            TRY(lb_allreduce(c, dst));
        else
            NCCL_CALL(c, c->comm, ncclAllReduce(dst, dst, 1, ncclDouble, ncclSum, c->comm, c->s), "err all-reduce");
        comm_mark(c, c->s, 2, 0, 0, (int64_t)sizeof(double));
        TRY(timed_end_on(c, c->s, e, MGP_TIMING_COLLECTIVE, (double)sizeof(double)));
    }
    update_metrics_old(c);
    return MGP_OK;
}

std::vector<char*> level_state(const mgp_ctx* c)
{
    std::vector<char*> v;
    for (const auto& L : c->lev) {
        v.push_back(L.u);
        v.push_back(L.t);
    }
    v.push_back(c->xbuf);
    return v;
}

void set_level_state(mgp_ctx* c, const std::vector<char*>& v)
{
    for (size_t l = 0; l < c->lev.size(); ++l) {
        c->lev[l].u = v[2 * l];
        c->lev[l].t = v[2 * l + 1];
    }
    c->xbuf = v[2 * c->lev.size()];
}

// Capture one cycle from the current buffer-pointer state into a new cache entry (nothing runs); the host
// state advances as if the cycle had run.
int capture_cycle(mgp_ctx* c, mgp_ctx::GraphEntry** out)
{
    const std::vector<char*> pre = level_state(c);
    HIP_TRY(c, hipStreamBeginCapture(c->s, hipStreamCaptureModeThreadLocal));
    const int rc = one_cycle(c, c->d_errs);  // err into d_errs[*d_slot] (mgp_cycles set err_ctr)
    hipGraph_t graph = nullptr;
    const hipError_t ec = hipStreamEndCapture(c->s, &graph);
    if (rc != MGP_OK) {
        if (graph) (void)hipGraphDestroy(graph);
        set_level_state(c, pre);
        return rc;
    }
    HIP_TRY(c, ec);
    mgp_ctx::GraphEntry e;
    e.pre = pre;
    e.post = level_state(c);
    const hipError_t ei = hipGraphInstantiate(&e.exec, graph, nullptr, nullptr, 0);
    (void)hipGraphDestroy(graph);
    HIP_TRY(c, ei);
    c->graphs.push_back(e);
    *out = &c->graphs.back();
    return MGP_OK;
}

// Capture the cycle graphs of every pointer state the cycle goes through (the finest level's buffers
// rotate with a period of 2 or 3 cycles) when the context is created, so that the first cycles replay
// back to back instead of idling the GPU during their captures.  The state ends where it began.
int precapture(mgp_ctx* c)
{
    const char* v = std::getenv("MGP_PRECAPTURE");
    if (!c->use_graph || c->handoff_fn || (v && std::atoi(v) == 0)) return MGP_OK;
    const std::vector<char*> s0 = level_state(c);
    c->err_ctr = c->o.err_mode && !c->multi() ? c->d_slot : nullptr;  // as mgp_cycles captures
    int rc = MGP_OK;
    for (int i = 0; i < 8 && rc == MGP_OK; ++i) {
        mgp_ctx::GraphEntry* e = nullptr;
        rc = capture_cycle(c, &e);
        if (rc == MGP_OK && e->post == s0) break;
    }
    c->err_ctr = nullptr;
    set_level_state(c, s0);
    c->metrics_old = nullptr;  // no outer iteration has run
    if (rc != MGP_OK) drop_graphs(c);
    return rc;
}

// One cycle through a cached hipGraph (captured on first use of a buffer-pointer state).
int graph_cycle(mgp_ctx* c, int slot)
{
    const std::vector<char*> pre = level_state(c);
    mgp_ctx::GraphEntry* hit = nullptr;
    for (auto& e : c->graphs)
        if (e.pre == pre) hit = &e;
    if (!hit) {
        if (c->graphs.size() >= 8) return one_cycle(c, c->d_errs);  // unusual state churn: eager
        TRY(capture_cycle(c, &hit));
    }
    set_level_state(c, hit->post);
    update_metrics_old(c);
    HIP_TRY(c, hipGraphLaunch(hit->exec, c->s));
    (void)slot;
    return MGP_OK;
}

void free_errs(mgp_ctx* c)
{
    if (c->errs_host && c->h_errs) (void)hipHostFree(c->h_errs);
    else if (c->d_errs) (void)hipFree(c->d_errs);
    c->d_errs = c->h_errs = nullptr;
    c->errs_host = false;
}

int ensure_errs(mgp_ctx* c, int k)
{
    if (k <= c->errs_cap) return MGP_OK;
    drop_graphs(c);  // captured graphs write into d_errs
    free_errs(c);
    int cap = std::max(k, 4096);
    if (c->errs_host_ok) {
        HIP_TRY(c, hipHostMalloc((void**)&c->h_errs, sizeof(double) * cap, hipHostMallocMapped | hipHostMallocCoherent));
        c->errs_host = true;
        HIP_TRY(c, hipHostGetDevicePointer((void**)&c->d_errs, c->h_errs, 0));
    } else {
        HIP_TRY(c, hipMalloc(&c->d_errs, sizeof(double) * cap));
    }
    c->errs_cap = cap;
    return MGP_OK;
}

int check_level(const mgp_ctx* c, int level)
{
    return (level >= 0 && level < (int)c->lev.size()) ? MGP_OK : MGP_ERR_ARG;
}

int sync_and_check(mgp_ctx* c)
{
    {
        // with peers, the stream may hold an exchange a failed rank never joins: the group may abort under it
        struct Wait {
            mgp_ctx* c;
            bool on;
            ~Wait()
            {
                if (on) c->waiting.fetch_sub(1);
            }
        } w{c, c->multi()};
        if (w.on) c->waiting.fetch_add(1);
        TRY(stream_wait(c, c->s));
        if (c->xs) TRY(stream_wait(c, c->xs));
    }
    if (c->stopped()) return c->fail(MGP_ERR_STATE, "%s", c->stop_msg());
    for (ncclComm_t comm : {c->comm, c->xcomm}) {
        if (!comm) continue;
        NcclScope scope(c);
        if (c->stopped()) return c->fail(MGP_ERR_STATE, "%s", c->stop_msg());
        ncclResult_t ar = ncclSuccess;
        NCCL_TRY(c, ncclCommGetAsyncError(comm, &ar));
        if (ar != ncclSuccess && ar != ncclInProgress)
            return c->fail(MGP_ERR_RCCL, "RCCL async error: %s", ncclGetErrorString(ar));
    }
    return MGP_OK;
}

}  // namespace

// =====================================================================================
// C ABI
// =====================================================================================
extern "C" {

int mgp_version(void) { return MGP_API_VERSION; }

void mgp_opts_default(mgp_opts* o)
{
    if (!o) return;
    std::memset(o, 0, sizeof(*o));
    o->struct_size = (int32_t)sizeof(mgp_opts);
    o->dim = 2;
    o->n[0] = o->n[1] = 8;
    o->n[2] = 1;
    o->real_bytes = 8;          // gpu.lua:32 picks double when the device has fp64
    o->nu1 = o->nu2 = 7;        // cpu.lua:20
    o->smoother = MGP_JACOBI;   // cpu.lua:57
    o->cycle = MGP_CYCLE_V;
    o->prolong = MGP_PROLONG_PC;
    o->coarse_init = MGP_COARSE_FRESH;
    o->coarse_bc = MGP_BC_ZERO;
    o->coarse_sweeps = 48;
    o->err_mode = 1;
    o->device = -1;
    o->rank = 0;
    o->world = 1;
    o->gather_cells = 32768;
    o->restriction = MGP_RESTRICT_AVERAGE;  // cpu.lua:127-135
    o->arith = MGP_ARITH_REAL;              // gpu.lua:32 (real-typed OpenCL arithmetic)
    o->api_version = MGP_API_VERSION;
}

int mgp_comm_unique_id(void* out, int64_t nbytes)
{
    if (!out || nbytes < (int64_t)sizeof(ncclUniqueId)) {
        g_create_error = "mgp_comm_unique_id: buffer too small";
        return MGP_ERR_ARG;
    }
    ncclUniqueId id;
    ncclResult_t r = ncclGetUniqueId(&id);
    if (r != ncclSuccess) {
        g_create_error = std::string("ncclGetUniqueId: ") + ncclGetErrorString(r);
        return MGP_ERR_RCCL;
    }
    std::memcpy(out, &id, sizeof(id));
    return MGP_OK;
}

static void select_engines(mgp_ctx* c);
static int level_engine(const mgp_ctx* c, int l);

// Everything mgp_create decides on the host before touching a device: options, the environment switches,
// ghost depth, the level hierarchy and each level's engine (shared with mgp_plan and mgp_plan_comm, so that
// those describe exactly what mgp_create would run).
static void host_setup(mgp_ctx* c, const mgp_opts& o, const std::vector<LevelPlan>& plan)
{
    c->o = o;
    if (c->o.dim == 2) c->o.n[2] = 1;
    c->rb = o.real_bytes;
    c->rk = real_kind(o);
    c->rccl1 = env_rccl1(o);
    {
        const char* v = std::getenv("MGP_COMM_TIMEOUT_S");  // (used by per-process RCCL contexts only: deadline_on)
        c->comm_timeout_s = v ? std::max(0.0, std::atof(v)) : 600.0;
        const char* vs = std::getenv("MGP_TEST_STALL");  // test hook: the k-th exchange holds its stream
        c->stall_at = vs ? std::max(0LL, std::atoll(vs)) : 0;
    }
    c->tu = mgp::fused_tuning_from_env();
    c->G = o.dim == 3 ? mgp::kGhost3D : 0;  // widened below when a distributed level is fused
    {
        const char* v = std::getenv("MGP_FRESH");
        c->fresh_sweep = !(v && std::atoi(v) == 0);
        const char* vb = std::getenv("MGP_POST_BLACK");
        c->post_black = !(vb && std::atoi(vb) == 0);
        const char* vp = std::getenv("MGP_POST1");
        c->post1 = vp && std::atoi(vp) != 0;
        const char* vd = std::getenv("MGP_DEEP_HALO");  // 0: exchange before every half-sweep instead
        c->deep_halo = !(vd && std::atoi(vd) == 0);
        const char* ve = std::getenv("MGP_EARLY_X");
        c->early_x = !(ve && std::atoi(ve) == 0);
        const char* vr = std::getenv("MGP_RESFW");
        c->resfw = !(vr && std::atoi(vr) == 0);
        const char* vbr = std::getenv("MGP_BRES");
        c->bres = !(vbr && std::atoi(vbr) == 0);
        const char* vrs = std::getenv("MGP_RBSWEEP");  // (measured slower, round 6: opt-in)
        c->rbsweep = vrs && std::atoi(vrs) != 0;
        const char* vb2 = std::getenv("MGP_BLK2");
        c->blk2 = !(vb2 && std::atoi(vb2) == 0);
        const char* veh = std::getenv("MGP_ERRS_HOST");
        c->errs_host_ok = !(veh && std::atoi(veh) == 0);
    }
    // distributed 3D levels sweep with deep halos (smooth_deep): kGhostZs ghost planes per side
    if (c->deep_halo && o.dim == 3 && c->multi()) c->G = mgp::kGhostZs;
    if (c->multi()) c->errs_host_ok = false;  // (the err all-reduce runs on d_errs)
    // MGP_PLANE_PAD (bytes, a multiple of 16; experiment): the plane stride of 3D levels with planes of >= 2^16 slots
    // is 2 H + pad instead of 2 H, so that equal cells of consecutive planes (which a z-streamed phase reads in the same
    // step) no longer share their address bits below the plane size
    const char* vpp = std::getenv("MGP_PLANE_PAD");
    const int64_t plane_pad = vpp ? (std::max(0LL, std::atoll(vpp)) & ~15LL) / c->rb : 0;
    for (auto& p : plan) {
        Level L;
        L.p = p;
        L.g = make_geo(p, c->o.dim);
        if (plane_pad && c->o.dim == 3 && L.g.P >= 65536) L.g.P += plane_pad;
        c->lev.push_back(L);
    }
    select_engines(c);
    for (auto& L : c->lev) L.alloc = L.g.P * (L.g.nz + 2 * c->G);
}

// the zero buffer of the lazily zeroed fresh coarse guesses: the largest such level's layout
static int64_t zbuf_reals_of(const mgp_ctx* c)
{
    int64_t z = 0;
    for (size_t l = 1; l < c->lev.size(); ++l)
        if (!c->lev[l].fused && (c->tail_level < 0 || (int)l < c->tail_level)) z = std::max(z, c->lev[l].alloc);
    return z;
}

int mgp_plan(const mgp_opts* o, int64_t* rows, int max_levels)
{
    if (!o) return MGP_ERR_ARG;
    std::vector<LevelPlan> plan;
    int rc = plan_levels(*o, plan, g_create_error);
    if (rc != MGP_OK) return rc;
    // the engines mgp_create would pick, on a device-free context
    mgp_ctx c;
    host_setup(&c, *o, plan);
    for (int l = 0; l < (int)plan.size() && l < max_levels && rows; ++l) {
        int64_t* r = rows + 8 * l;
        r[0] = plan[l].nx;
        r[1] = plan[l].ny;
        r[2] = plan[l].gnz;
        r[3] = plan[l].nz;
        r[4] = plan[l].z0;
        r[5] = plan[l].dist;
        r[6] = level_engine(&c, l);
        r[7] = 0;
    }
    return (int)plan.size();
}


// level 0's u and f were just written (init or host I/O): their ghost planes are stale on a slab level
static void fields_written(mgp_ctx* c)
{
    Level& L = c->lev[0];
    L.ghost_ok = !L.p.dist;
    L.ghost_zero = false;
    L.fghost_ok = !L.p.dist;
}

int mgp_plan_comm(const mgp_opts* o, int32_t cycles, int64_t* rows, int max_rows)
{
    if (!o || cycles < 0 || max_rows < 0 || (max_rows > 0 && !rows)) return MGP_ERR_ARG;
    std::vector<LevelPlan> plan;
    int rc = plan_levels(*o, plan, g_create_error);
    if (rc != MGP_OK) return rc;
    mgp_ctx c;
    host_setup(&c, *o, plan);
    c.dry = true;
    // stand-ins for the device objects whose presence steers the host logic (never dereferenced: every device
    // call is skipped): the side stream of the early exchange and the zero buffer of lazily zeroed levels
    static char stand_in[16];
    if (c.multi() && c.early_x) c.xs = reinterpret_cast<hipStream_t>(stand_in);
    if (c.o.smoother == MGP_RBGS && c.o.coarse_init == MGP_COARSE_FRESH) {
        c.zbuf_reals = zbuf_reals_of(&c);
        if (c.zbuf_reals) c.zbuf = stand_in;
    }
    fields_written(&c);  // after mgp_init_point_charge (or mgp_set_field) of psi and f
    for (int k = 0; k < cycles; ++k) {
        rc = one_cycle(&c, nullptr);
        if (rc != MGP_OK) {
            g_create_error = c.err;
            return rc;
        }
    }
    c.xs = nullptr;
    c.zbuf = nullptr;
    return mgp_comm_log(&c, rows, max_rows, 0);
}

static void destroy_impl(mgp_ctx* c)
{
    if (!c) return;
    if (c->stall_flag) __atomic_store_n(c->stall_flag, 1, __ATOMIC_RELEASE);
    if (c->s) (void)hipStreamSynchronize(c->s);
    for (auto& L : c->lev) {
        if (L.u) dev_free(c, L.u);
        if (L.f) dev_free(c, L.f);
        if (L.t) dev_free(c, L.t);
    }
    if (c->zbuf) (void)hipFree(c->zbuf);
    if (c->psi_old) (void)hipFree(c->psi_old);
    if (c->rscratch) (void)hipFree(c->rscratch);
    if (c->xbuf) dev_free(c, c->xbuf);
    if (c->stage) (void)hipFree(c->stage);
    if (c->d_stats_h) (void)hipFree(c->d_stats_h);
    if (c->d_part) (void)hipFree(c->d_part);
    free_errs(c);
    if (c->d_err_cur) (void)hipFree(c->d_err_cur);
    if (c->d_slot) (void)hipFree(c->d_slot);
    for (auto& g : c->graphs) (void)hipGraphExecDestroy(g.exec);
    for (auto e : c->ev) (void)hipEventDestroy(e);
    if (c->xcomm) (void)ncclCommDestroy(c->xcomm);
    if (c->comm) (void)ncclCommDestroy(c->comm);
    if (c->lb) {
        std::lock_guard<std::mutex> lk(c->lb->m);
        if (c->o.rank >= 0 && c->o.rank < (int)c->lb->ranks.size() && c->lb->ranks[c->o.rank] == c)
            c->lb->ranks[c->o.rank] = nullptr;
    }
    if (c->lb_ev) (void)hipEventDestroy(c->lb_ev);
    if (c->lb_ev2) (void)hipEventDestroy(c->lb_ev2);
    if (c->xs) (void)hipStreamSynchronize(c->xs);
    if (c->x_ev0) (void)hipEventDestroy(c->x_ev0);
    if (c->x_ev1) (void)hipEventDestroy(c->x_ev1);
    if (c->xs) (void)hipStreamDestroy(c->xs);
    if (c->lb_red) (void)hipFree(c->lb_red);
    if (c->d_metrics) (void)hipFree(c->d_metrics);
    if (c->d_rn) (void)hipFree(c->d_rn);
    if (c->d_dbg) (void)hipFree(c->d_dbg);
    for (auto& m : c->marks)
        if (m.ev) (void)hipEventDestroy(m.ev);
    if (c->stall_flag) (void)hipHostFree(c->stall_flag);
    if (c->s) (void)hipStreamDestroy(c->s);
    delete c;
}

static int create_impl(mgp_ctx** out, const mgp_opts* o, mgp_loopback* lb, ncclComm_t comm = nullptr,
                       ncclComm_t xcomm = nullptr);

int mgp_create(mgp_ctx** out, const mgp_opts* o) { return create_impl(out, o, nullptr); }

int mgp_loopback_create(mgp_loopback** out, int world)
{
    if (!out || world < 1) return MGP_ERR_ARG;
    mgp_loopback* g = new mgp_loopback();
    g->world = world;
    g->ranks.assign((size_t)world, nullptr);
    *out = g;
    return MGP_OK;
}

void mgp_loopback_destroy(mgp_loopback* lb) { delete lb; }

int mgp_create_loopback(mgp_ctx** out, const mgp_opts* o, mgp_loopback* lb)
{
    if (!lb || !o || o->world != lb->world) {
        g_create_error = "mgp_create_loopback: group size != opts.world";
        return MGP_ERR_ARG;
    }
    return create_impl(out, o, lb);
}

// How each level's phases run (host logic only, no device): the temporally blocked phases (k_zs),
// the tiled one-launch phases (k_blk) and the one-launch coarse tail; shared by mgp_create and mgp_plan.
static void select_engines(mgp_ctx* c)
{
    if (c->rk == mgp::kRealF32D) {
        // cpu-raw.lua's float arithmetic (cpu-raw.lua:142-153, 186-237): every level one launch per piece through
        // the scalar double-evaluating kernels; the err is calcFrobErr's float errorBuf summed after the cycle
        // (cpu-raw.lua:249-254); the fused, tiled and tail engines evaluate in the real type and stay off
        c->err_fuse = false;
        c->fresh_sweep = false;
        c->post1 = false;
        for (auto& L : c->lev) L.fused = L.blk = L.zpost = false;
        c->tail_level = -1;
        return;
    }
    c->err_fuse = c->o.err_mode && c->o.smoother == MGP_RBGS && c->o.nu1 >= 1 && c->o.nu2 >= 1 && c->lev.size() > 1;
    {
        // temporally blocked phases: RB-GS 2+2 on 3D levels of >= MGP_FUSED_MIN_CELLS cells per rank (k_zs,
        // default 2^25) and on 2D levels of >= MGP_YS_MIN_CELLS cells (k_ys, default 2^24); MGP_FUSED=0 turns
        // them off (one launch per half-sweep, bit-identical results).  A distributed fused level exchanges
        // kGhostZs-deep halos, so every level gets that many ghost planes.
        const char* v = std::getenv("MGP_FUSED");
        const char* vm = std::getenv(c->o.dim == 2 ? "MGP_YS_MIN_CELLS" : "MGP_FUSED_MIN_CELLS");
        // (2D: 4096^2 measured 0.285 ms per cycle with only level 0 streamed, 0.406 with 2048^2 as well)
        const int64_t min_cells = vm ? std::atoll(vm) : (int64_t(1) << (c->o.dim == 2 ? 24 : 25));
        const bool on = !(v && std::atoi(v) == 0) && c->o.smoother == MGP_RBGS && c->o.nu1 == 2 && c->o.nu2 == 2;
        for (size_t l = 0; l + 1 < c->lev.size(); ++l) {
            Level& L = c->lev[l];
            L.fused = on && level_cells(L) >= min_cells && mgp::fused_supported(c->rb, c->o.dim, 2, L.g, c->tu);
            if (L.fused) {
                const bool clz = coarse_coef(c->o.coarse_bc, (int)l) == 0.0;
                L.zc = mgp::fused_zc(c->rb, L.g, false, clz, c->tu);
                L.zc_pre = mgp::fused_zc(c->rb, L.g, true, clz, c->tu);
            }
            if (L.fused && L.p.dist) c->G = mgp::kGhostZs;
        }
        // POST alone temporally blocked on the 3D levels of >= MGP_ZPOST_MIN_CELLS cells (default 2^24) below that:
        // at 256^3 (cl != 0) k_zs POST takes 66 us against 84 us for the prolongation + 4 half-sweeps, while
        // its PRE (109 us + a 10 us fill of the fresh guess) loses to the per-piece 94 us
        const char* vz = std::getenv("MGP_ZPOST_MIN_CELLS");
        const int64_t zmin = vz ? std::atoll(vz) : (c->o.dim == 3 ? int64_t(1) << 24 : INT64_MAX);
        for (size_t l = 1; l + 1 < c->lev.size(); ++l) {
            Level& L = c->lev[l];
            L.zpost = on && !L.fused && level_cells(L) >= zmin && mgp::fused_supported(c->rb, c->o.dim, 2, L.g, c->tu);
            if (L.zpost) L.zc = mgp::fused_zc(c->rb, L.g, false, coarse_coef(c->o.coarse_bc, (int)l) == 0.0, c->tu);
            if (L.zpost && L.p.dist) c->G = mgp::kGhostZs;
        }
    }
    {
        // tiled one-launch phases (k_blk) on replicated RB-GS levels 1 .. of <= MGP_BLK_CELLS cells
        // below the finest; MGP_BLK=0 turns them off (bit-identical results)
        const char* v = std::getenv("MGP_BLK");
        const char* vm = std::getenv("MGP_BLK_CELLS");
        // defaults measured: 3D 64^3 (128^3 measured slower than one launch per piece), 2D 1024^2
        const int64_t max_cells = vm ? std::atoll(vm) : (int64_t(1) << (c->o.dim == 3 ? 18 : 20));
        const int ns = std::max(c->o.nu1, c->o.nu2);
        const bool on = !(v && std::atoi(v) == 0) && c->o.smoother == MGP_RBGS && c->o.nu1 >= 1 && c->o.nu2 >= 1;
        for (size_t l = 1; l + 1 < c->lev.size(); ++l) {
            Level& L = c->lev[l];
            L.blk = on && !L.fused && !L.zpost && !L.p.dist && level_cells(L) <= max_cells &&
                    mgp::block_supported(c->rb, c->o.dim, ns, L.g);
        }
    }
    plan_tail(c);
}

// mgp_level_info / mgp_plan engine code: 0 one launch per piece, 1 coarse tail, 2 k_zs, 3 k_blk, 4 PRE per
// piece + k_zs POST
static int level_engine(const mgp_ctx* c, int l)
{
    const Level& L = c->lev[l];
    return c->tail_level >= 0 && l >= c->tail_level ? 1 : L.fused ? 2 : L.blk ? 3 : L.zpost ? 4 : 0;
}

static int create_impl(mgp_ctx** out, const mgp_opts* o, mgp_loopback* lb, ncclComm_t ext_comm, ncclComm_t ext_xcomm)
{
    if (!out || !o) {
        g_create_error = "mgp_create: null argument";
        return MGP_ERR_ARG;
    }
    *out = nullptr;
    std::vector<LevelPlan> plan;
    int rc = plan_levels(*o, plan, g_create_error);
    if (rc != MGP_OK) return rc;

    mgp_ctx* c = new mgp_ctx();
    if (ext_comm) {  // from mgp_group_create (non-blocking communicators); owned from here
        c->comm = ext_comm;
        c->xcomm = ext_xcomm;
        c->nb_comm = true;
    }
    host_setup(c, *o, plan);
    auto bail = [&](int code) {
        g_create_error = c->err;
        destroy_impl(c);
        return code;
    };
    int ndev = 0;
    hipError_t he = hipGetDeviceCount(&ndev);
    if (he != hipSuccess || ndev == 0) {
        c->err = std::string("no HIP device available: ") + hipGetErrorString(he);
        return bail(MGP_ERR_HIP);
    }
    if (o->device >= 0) {
        if (o->device >= ndev) {
            c->err = "device ordinal out of range";
            return bail(MGP_ERR_ARG);
        }
        he = hipSetDevice(o->device);
        if (he != hipSuccess) {
            c->err = std::string("hipSetDevice: ") + hipGetErrorString(he);
            return bail(MGP_ERR_HIP);
        }
    }
    (void)hipGetDevice(&c->device);
    he = hipStreamCreateWithFlags(&c->s, hipStreamNonBlocking);
    if (he != hipSuccess) {
        c->err = std::string("hipStreamCreate: ") + hipGetErrorString(he);
        return bail(MGP_ERR_HIP);
    }
    const size_t rb = (size_t)c->rb;
    c->pad = pad_bytes();
    for (size_t l = 0; l < c->lev.size(); ++l) {
        Level& L = c->lev[l];
        const size_t bytes = (size_t)L.alloc * rb;
        const bool need_t = c->o.smoother == MGP_JACOBI || (l == 0 && c->err_fuse) || L.fused || L.blk || L.zpost ||
                            rbsweep_level(c, L, (int)l);
        if (dev_alloc(c, &L.u, bytes, 1) != hipSuccess || dev_alloc(c, &L.f, bytes, 2) != hipSuccess ||
            (need_t && dev_alloc(c, &L.t, bytes, 3) != hipSuccess)) {
            c->err = "hipMalloc failed for level " + std::to_string(l) + " (" + std::to_string(bytes) + " bytes)";
            return bail(MGP_ERR_OOM);
        }
        // zero everything once: physical ghost planes stay 0 for the context's lifetime
        if (hipMemsetAsync(L.u, 0, bytes, c->s) != hipSuccess || hipMemsetAsync(L.f, 0, bytes, c->s) != hipSuccess ||
            (need_t && hipMemsetAsync(L.t, 0, bytes, c->s) != hipSuccess)) {
            c->err = "hipMemset failed";
            return bail(MGP_ERR_HIP);
        }
    }
    const Level& L0 = c->lev[0];
    const size_t interior = (size_t)(L0.g.P * L0.g.nz) * rb;
    if (c->o.err_mode && !c->err_fuse && hipMalloc(&c->psi_old, interior) != hipSuccess) {
        c->err = "hipMalloc failed for psiOld";
        return bail(MGP_ERR_OOM);
    }
    {
        const char* v = std::getenv("MGP_KEEP_PSI_OLD");
        if (c->o.err_mode && c->err_fuse && L0.fused && !(v && std::atoi(v) == 0)) {
            if (dev_alloc(c, &c->xbuf, (size_t)L0.alloc * rb, 4) != hipSuccess ||
                hipMemsetAsync(c->xbuf, 0, (size_t)L0.alloc * rb, c->s) != hipSuccess) {
                c->err = "hipMalloc failed for the psiOld-keeping output buffer";
                return bail(MGP_ERR_OOM);
            }
        }
    }
    // the full weighting reads residuals of neighbouring coarse cells' children: r is materialised once per
    // level in this scratch (level 0 is the largest level; the kernels never read its physical ghost planes)
    if (ensure_rscratch(c, true) != MGP_OK) return bail(MGP_ERR_OOM);
    {
        // staging for host I/O: at least one level-0 plane, at most ~256 MiB (or the whole interior)
        const size_t plane = (size_t)(L0.p.nx * L0.p.ny) * rb;
        c->stage_bytes = std::min(interior, std::max(plane, (size_t)256 << 20));
        if (hipMalloc(&c->stage, c->stage_bytes) != hipSuccess ||
            hipMalloc(&c->d_stats_h, sizeof(uint64_t) * (mgp::kSumBlocks + 1) + sizeof(double) * (3 * mgp::kSumBlocks + 3)) !=
                hipSuccess) {
            c->err = "hipMalloc failed for the staging buffer";
            return bail(MGP_ERR_OOM);
        }
    }
    {
        const char* v = std::getenv("MGP_GS");
        c->use_gs = v && std::atoi(v) != 0;
    }
    int nb2 = 2 * mgp::half_blocks(c->rk, L0.g, c->use_gs);
    if (L0.fused) nb2 = std::max(nb2, mgp::fused_blocks(c->rb, L0.g, L0.zc, coarse_coef(c->o.coarse_bc, 0) == 0.0, c->tu));
    c->part_cap = std::max<int64_t>(mgp::kSumBlocks, nb2 + mgp::sum_scratch(nb2));
    if (hipMalloc(&c->d_part, sizeof(double) * c->part_cap) != hipSuccess) {
        c->err = "hipMalloc failed for reduction partials";
        return bail(MGP_ERR_OOM);
    }
    if (ensure_errs(c, 64) != MGP_OK || hipMalloc(&c->d_err_cur, sizeof(double)) != hipSuccess ||
        hipMalloc(&c->d_slot, sizeof(int)) != hipSuccess) {
        c->err = "hipMalloc failed for err slots";
        return bail(MGP_ERR_OOM);
    }
    {
        const char* v = std::getenv("MGP_GRAPH");
        c->use_graph = !c->multi() && !(v && std::atoi(v) == 0) && !roctx_on();
    }
    if (c->o.smoother == MGP_RBGS && c->o.coarse_init == MGP_COARSE_FRESH) {
        c->zbuf_reals = zbuf_reals_of(c);
        const size_t zb = (size_t)c->zbuf_reals * rb;
        if (zb && (hipMalloc(&c->zbuf, zb) != hipSuccess || hipMemsetAsync(c->zbuf, 0, zb, c->s) != hipSuccess)) {
            c->err = "hipMalloc failed for the zero buffer";
            return bail(MGP_ERR_OOM);
        }
        const char* v = std::getenv("MGP_LAZY_ZERO");  // 0: memset every fresh coarse guess instead
        if (v && std::atoi(v) == 0) c->lazy_zero = false;
        const char* vf = std::getenv("MGP_LAZY_ZERO_FUSED");
        if (vf && std::atoi(vf) == 0) c->lazy_zero_fused = false;
    }
    he = mgp::prepare_kernels(c->rb);
    if (he != hipSuccess) {
        c->err = std::string("hipFuncSetAttribute (dynamic LDS): ") + hipGetErrorString(he);
        return bail(MGP_ERR_HIP);
    }
    if (c->multi()) {  // side stream of the early POST halo exchange
        if (c->early_x && (hipStreamCreateWithFlags(&c->xs, hipStreamNonBlocking) != hipSuccess ||
                           hipEventCreateWithFlags(&c->x_ev0, hipEventDisableTiming) != hipSuccess ||
                           hipEventCreateWithFlags(&c->x_ev1, hipEventDisableTiming) != hipSuccess)) {
            c->err = "exchange stream setup failed";
            return bail(MGP_ERR_HIP);
        }
    }
    if (c->o.world > 1 && lb) {
        c->lb = lb;
        if (hipEventCreateWithFlags(&c->lb_ev, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&c->lb_ev2, hipEventDisableTiming) != hipSuccess ||
            hipMalloc(&c->lb_red, sizeof(double) * 3 * c->o.world) != hipSuccess) {
            c->err = "loopback transport setup failed";
            c->lb = nullptr;
            return bail(MGP_ERR_HIP);
        }
        std::lock_guard<std::mutex> lk(lb->m);
        if (lb->ranks[c->o.rank]) {
            c->err = "loopback rank already registered";
            c->lb = nullptr;
            return bail(MGP_ERR_ARG);
        }
        lb->ranks[c->o.rank] = c;
    } else if (c->multi() && c->comm) {
        // communicator handed in by mgp_group_create
    } else if (c->multi()) {
        ncclUniqueId id;
        std::memcpy(&id, o->comm_id, sizeof(id));
        if (c->rccl1) {  // one rank: its own id
            const ncclResult_t ri = ncclGetUniqueId(&id);
            if (ri != ncclSuccess) {
                c->err = std::string("ncclGetUniqueId: ") + ncclGetErrorString(ri);
                return bail(MGP_ERR_RCCL);
            }
        }
        ncclResult_t r = ncclCommInitRank(&c->comm, c->o.world, id, c->o.rank);
        if (r != ncclSuccess) {
            c->err = std::string("ncclCommInitRank: ") + ncclGetErrorString(r);
            c->comm = nullptr;
            return bail(MGP_ERR_RCCL);
        }
        // the side stream's communicator: a collective split that every rank makes at this point, whatever its
        // environment says (MGP_EARLY_X only decides whether it is used), so that the early POST
        // exchange does not serialise with the compute stream's exchanges of the coarse levels
        r = ncclCommSplit(c->comm, 0, c->o.rank, &c->xcomm, nullptr);
        if (r != ncclSuccess) {
            c->err = std::string("ncclCommSplit (side-stream communicator): ") + ncclGetErrorString(r);
            c->xcomm = nullptr;
            return bail(MGP_ERR_RCCL);
        }
    }
    if (c->stall_at && c->deadline_on()) {  // (test hook MGP_TEST_STALL) the flag that releases the held stream
        if (hipHostMalloc((void**)&c->stall_flag, sizeof(int), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
            hipHostGetDevicePointer((void**)&c->stall_flag_d, c->stall_flag, 0) != hipSuccess) {
            c->err = "MGP_TEST_STALL: no pinned flag";
            return bail(MGP_ERR_HIP);
        }
        *c->stall_flag = 0;
    }
    if (hipStreamSynchronize(c->s) != hipSuccess) {
        c->err = "stream synchronisation after allocation failed";
        return bail(MGP_ERR_HIP);
    }
    if (precapture(c) != MGP_OK) return bail(MGP_ERR_HIP);
    *out = c;
    return MGP_OK;
}

void mgp_destroy(mgp_ctx* c) { destroy_impl(c); }

const char* mgp_last_error(const mgp_ctx* c) { return c ? c->err.c_str() : g_create_error.c_str(); }

int mgp_num_levels(const mgp_ctx* c) { return c ? (int)c->lev.size() : MGP_ERR_ARG; }

int mgp_level_info(const mgp_ctx* c, int level, int64_t info[8])
{
    if (!c || !info || check_level(c, level) != MGP_OK) return MGP_ERR_ARG;
    const LevelPlan& p = c->lev[level].p;
    info[0] = p.nx;
    info[1] = p.ny;
    info[2] = p.gnz;
    info[3] = p.nz;
    info[4] = p.z0;
    info[5] = p.dist;
    info[6] = level_engine(c, level);
    info[7] = c->lev[level].exchanges;
    return MGP_OK;
}

int mgp_init_point_charge(mgp_ctx* c)
{
    if (!c) return MGP_ERR_ARG;
    Level& L = c->lev[0];
    const int64_t cz = c->o.dim == 3 ? L.p.gnz / 2 : 0;
    HIP_TRY(c, mgp::launch_init_point_charge(c->rb, c->o.dim, c->ui(L, L.u), c->ui(L, L.f), L.g, L.p.nx / 2,
                                             L.p.ny / 2, cz, c->s));
    fields_written(c);
    return sync_and_check(c);
}


// Host <-> packed level I/O in plane chunks through the bounded staging buffer (a 4096 x 4096 x 512
// slab is 34 GB per field; no full-size staging copy is ever allocated).
// The packed buffer a read of `which` comes from: stored fields directly, computed views into a
// temporary level-sized buffer (*scratch, freed by the caller).
static int field_source(mgp_ctx* c, int level, int which, char** src, char** scratch)
{
    Level& L = c->lev[(size_t)level];
    *scratch = nullptr;
    switch (which) {
    case MGP_FIELD_U: *src = L.u; return MGP_OK;
    case MGP_FIELD_F: *src = L.f; return MGP_OK;
    case MGP_FIELD_TMP:
        if (!L.t) return c->fail(MGP_ERR_STATE, "tmpU: level %d has no second buffer (in-place red/black GS)", level);
        *src = L.t;
        return MGP_OK;
    case MGP_FIELD_PSI_OLD:
    case MGP_FIELD_ERROR:
        if (level != 0 || !c->metrics_old)
            return c->fail(MGP_ERR_STATE, "psiOld / errorBuf: level 0 only, after an outer iteration with err_mode 1 "
                                          "that kept psiOld (not with MGP_KEEP_PSI_OLD=0 on the temporally blocked finest level)");
        break;
    case MGP_FIELD_CORRECTION:
        if (level + 1 >= (int)c->lev.size()) return c->fail(MGP_ERR_ARG, "vs: the coarsest level has none");
        break;
    case MGP_FIELD_RESIDUAL: break;
    default: return c->fail(MGP_ERR_ARG, "unknown field %d", which);
    }
    const size_t bytes = (size_t)L.alloc * c->rb;
    if (hipMalloc(scratch, bytes) != hipSuccess) return c->fail(MGP_ERR_OOM, "no room for a computed field view");
    HIP_TRY(c, hipMemsetAsync(*scratch, 0, bytes, c->s));
    char* sc = c->ui(L, *scratch);
    const int64_t n = L.g.P * L.g.nz;
    if (which == MGP_FIELD_PSI_OLD) {
        HIP_TRY(c, hipMemcpyAsync(sc, c->metrics_old, (size_t)n * c->rb, hipMemcpyDeviceToDevice, c->s));
    } else if (which == MGP_FIELD_ERROR) {
        HIP_TRY(c, mgp::launch_sqdiff_field(c->rk, c->ui(L, L.u), c->metrics_old, sc, n, c->s));
    } else if (which == MGP_FIELD_RESIDUAL) {
        TRY(exchange(c, L));
        HIP_TRY(c, mgp::launch_residual_field(c->rk, c->o.dim, c->ui(L, L.u), c->ui(L, L.f), sc, L.g, level_h(c, level),
                                              coarse_coef(c->o.coarse_bc, level), c->s));
    } else {  // MGP_FIELD_CORRECTION: P V onto zeros
        Level& C = c->lev[(size_t)level + 1];
        TRY(materialize_zero(c, C));
        const int linear = c->o.prolong == MGP_PROLONG_LINEAR;
        if (linear && C.p.dist) TRY(exchange(c, C));
        int64_t zc = 0;
        const Geo gc = coarse_view(L, C, &zc);
        char* V = c->ui(C, C.u) + (size_t)(zc * C.g.P) * c->rb;
        HIP_TRY(c, mgp::launch_prolong_correct(c->rk, c->o.dim, linear, sc, V, L.g, gc,
                                               coarse_coef(c->o.coarse_bc, level + 1), c->s));
    }
    *src = *scratch;
    return MGP_OK;
}

// Host <-> packed level I/O in plane chunks through the bounded staging buffer (a 4096 x 4096 x 512
// slab is 34 GB per field; no full-size staging copy is ever allocated).
static int planes_io(mgp_ctx* c, int level, int which, int64_t z_begin, int64_t nz, void* buf, int mem, bool to_device)
{
    if (check_level(c, level) != MGP_OK || which < 0 || which >= MGP_FIELD_KINDS || !buf)
        return c->fail(MGP_ERR_ARG, "field I/O: bad level / field / buffer");
    if (to_device && which != MGP_FIELD_U && which != MGP_FIELD_F)
        return c->fail(MGP_ERR_ARG, "field %d is a read-only view", which);
    Level& L = c->lev[level];
    if (z_begin < 0 || nz < 0 || z_begin + nz > L.g.nz)
        return c->fail(MGP_ERR_ARG, "field I/O: planes [%lld, %lld) outside the local slab of %lld planes",
                       (long long)z_begin, (long long)(z_begin + nz), (long long)L.g.nz);
    WaitScope wait(c);  // a derived field may exchange halos first, and the read-back waits for that
    if (which == MGP_FIELD_U || which == MGP_FIELD_RESIDUAL) TRY(materialize_zero(c, L));
    char* src = nullptr;
    char* scratch = nullptr;
    if (to_device) {
        src = which == MGP_FIELD_U ? L.u : L.f;
    } else {
        const int rc = field_source(c, level, which, &src, &scratch);
        if (rc != MGP_OK) {
            if (scratch) (void)hipFree(scratch);
            return rc;
        }
    }
    struct Free {
        char* p;
        ~Free() { if (p) (void)hipFree(p); }
    } free_scratch{scratch};
    char* base = c->ui(L, src);
    const size_t rb = (size_t)c->rb;
    const int64_t lex_plane = L.p.nx * L.p.ny;  // reals per plane, lexicographic
    const int64_t per_chunk =
        mem == MGP_MEM_DEVICE ? nz : std::max<int64_t>(1, (int64_t)(c->stage_bytes / (lex_plane * rb)));
    for (int64_t z = z_begin; z < z_begin + nz; z += per_chunk) {
        const int64_t cn = std::min(per_chunk, z_begin + nz - z);
        Geo gs = L.g;
        gs.nz = cn;
        gs.z0 = L.g.z0 + z;
        char* packed = base + (size_t)(z * L.g.P) * rb;
        char* hb = (char*)buf + (size_t)((z - z_begin) * lex_plane) * rb;
        const size_t bytes = (size_t)(cn * lex_plane) * rb;
        if (to_device) {
            const void* lex = hb;
            if (mem != MGP_MEM_DEVICE) {
                HIP_TRY(c, hipMemcpyAsync(c->stage, hb, bytes, hipMemcpyHostToDevice, c->s));
                lex = c->stage;
            }
            HIP_TRY(c, mgp::launch_pack(c->rb, lex, packed, gs, c->s));
        } else {
            void* lex = mem == MGP_MEM_DEVICE ? (void*)hb : (void*)c->stage;
            HIP_TRY(c, mgp::launch_unpack(c->rb, packed, lex, gs, c->s));
            if (mem != MGP_MEM_DEVICE) {
                HIP_TRY(c, hipMemcpyAsync(hb, c->stage, bytes, hipMemcpyDeviceToHost, c->s));
                TRY(stream_wait(c, c->s));  // the next chunk reuses the staging buffer
            }
        }
    }
    if (to_device) {
        if (which == MGP_FIELD_U) {
            L.ghost_ok = !L.p.dist;
            L.ghost_zero = false;
        } else {
            L.fghost_ok = !L.p.dist;
        }
    }
    return sync_and_check(c);
}

int mgp_set_field(mgp_ctx* c, int level, int which, const void* src, int64_t count, int mem)
{
    if (!c) return MGP_ERR_ARG;
    if (check_level(c, level) != MGP_OK) return c->fail(MGP_ERR_ARG, "mgp_set_field: bad level %d", level);
    Level& L = c->lev[level];
    if (count != level_count(L))
        return c->fail(MGP_ERR_ARG, "mgp_set_field: count %lld != %lld", (long long)count, (long long)level_count(L));
    return planes_io(c, level, which, 0, L.g.nz, const_cast<void*>(src), mem, true);
}

int mgp_get_field(const mgp_ctx* cc, int level, int which, void* dst, int64_t count, int mem)
{
    mgp_ctx* c = const_cast<mgp_ctx*>(cc);
    if (!c) return MGP_ERR_ARG;
    if (check_level(c, level) != MGP_OK) return c->fail(MGP_ERR_ARG, "mgp_get_field: bad level %d", level);
    Level& L = c->lev[level];
    if (count != level_count(L))
        return c->fail(MGP_ERR_ARG, "mgp_get_field: count %lld != %lld", (long long)count, (long long)level_count(L));
    return planes_io(c, level, which, 0, L.g.nz, dst, mem, false);
}

int mgp_set_planes(mgp_ctx* c, int level, int which, int64_t z_begin, int64_t nz, const void* src, int mem)
{
    if (!c) return MGP_ERR_ARG;
    return planes_io(c, level, which, z_begin, nz, const_cast<void*>(src), mem, true);
}

int mgp_get_planes(const mgp_ctx* cc, int level, int which, int64_t z_begin, int64_t nz, void* dst, int mem)
{
    mgp_ctx* c = const_cast<mgp_ctx*>(cc);
    if (!c) return MGP_ERR_ARG;
    return planes_io(c, level, which, z_begin, nz, dst, mem, false);
}

int mgp_field_stats(const mgp_ctx* cc, int level, int which, uint64_t* hash, double stats[3])
{
    mgp_ctx* c = const_cast<mgp_ctx*>(cc);
    if (!c) return MGP_ERR_ARG;
    if (check_level(c, level) != MGP_OK || (which != MGP_FIELD_U && which != MGP_FIELD_F))
        return c->fail(MGP_ERR_ARG, "mgp_field_stats: bad level / field");
    Level& L = c->lev[level];
    if (which == MGP_FIELD_U) TRY(materialize_zero(c, L));
    uint64_t* hp = c->d_stats_h;
    double* dp = (double*)(hp + mgp::kSumBlocks + 1);
    HIP_TRY(c, mgp::launch_field_stats(c->rb, c->ui(L, which == MGP_FIELD_U ? L.u : L.f), L.g, hp, dp,
                                       hp + mgp::kSumBlocks, dp + 3 * mgp::kSumBlocks, c->s));
    uint64_t h = 0;
    double d[3];
    HIP_TRY(c, hipMemcpyAsync(&h, hp + mgp::kSumBlocks, sizeof h, hipMemcpyDeviceToHost, c->s));
    HIP_TRY(c, hipMemcpyAsync(d, dp + 3 * mgp::kSumBlocks, sizeof d, hipMemcpyDeviceToHost, c->s));
    TRY(sync_and_check(c));
    if (hash) *hash = h;
    if (stats) std::memcpy(stats, d, sizeof d);
    return MGP_OK;
}

int mgp_cycles(mgp_ctx* c, int32_t k, double* errs)
{
    if (!c || k < 0) return MGP_ERR_ARG;
    TRY(ensure_errs(c, k));
    const bool graph = c->use_graph && !c->timing && !c->handoff_fn && !c->debug;
    // one GPU: every cycle's err goes to d_errs[*d_slot] and advances the device counter (graph replays
    // need no per-cycle copy); with ranks the all-reduce needs the slot's address, so it is explicit
    const bool ctr = !c->multi() && c->o.err_mode && k > 0;
    if (ctr) HIP_TRY(c, hipMemsetAsync(c->d_slot, 0, sizeof(int), c->s));
    c->err_ctr = ctr ? c->d_slot : nullptr;
    if (c->debug) {
        c->dbg_names.clear();
        HIP_TRY(c, hipMemsetAsync(c->d_dbg, 0x7f, sizeof(int), c->s));
    }
    int rc = MGP_OK;
    for (int i = 0; i < k && rc == MGP_OK; ++i) {
        c->dbg_cycle = i + 1;
        rc = graph ? graph_cycle(c, i) : one_cycle(c, ctr ? c->d_errs : c->d_errs + i);
    }
    c->err_ctr = nullptr;
    TRY(rc);
    TRY(sync_and_check(c));
    if (c->debug) {
        int first = 0;
        HIP_TRY(c, hipMemcpy(&first, c->d_dbg, sizeof(int), hipMemcpyDeviceToHost));
        if (first >= 0 && first < (int)c->dbg_names.size()) {
            c->fail_after_sync = true;
            return c->fail(MGP_ERR_STATE, "found a nan (cpu-raw.lua:135-139, gpu.lua:279-283): %s",
                           c->dbg_names[(size_t)first].c_str());
        }
    }
    if (errs) {
        if (!c->o.err_mode) {
            for (int i = 0; i < k; ++i) errs[i] = NAN;
        } else {
            std::vector<double> sums((size_t)k);
            if (c->errs_host)
                std::memcpy(sums.data(), c->h_errs, sizeof(double) * k);  // (coherent, after the stream sync)
            else
                HIP_TRY(c, hipMemcpy(sums.data(), c->d_errs, sizeof(double) * k, hipMemcpyDeviceToHost));
            const double n = (double)c->ncells_global();
            for (int i = 0; i < k; ++i) errs[i] = std::sqrt(sums[i] / n);  // cpu.lua:203
        }
    }
    return MGP_OK;
}

int mgp_cycle(mgp_ctx* c, double* err_out)
{
    double e = NAN;
    int rc = mgp_cycles(c, 1, &e);
    if (err_out) *err_out = e;
    return rc;
}

int mgp_two_grid(mgp_ctx* c, double h, void* u, const void* f, int64_t L, int mem)
{
    if (!c || !u || !f) return MGP_ERR_ARG;
    if (c->o.world > 1) return c->fail(MGP_ERR_STATE, "mgp_two_grid: single-GPU contexts only");
    for (int l = 0; l < (int)c->lev.size(); ++l) {
        Level& Lv = c->lev[l];
        if (Lv.p.nx != L) continue;
        // twoGrid(h, u, f, L) works on the caller's buffers (cpu-raw.lua:186, gpu.lua:296): the level's
        // own u / f (on level 0 the solver's psi and RHS) are saved and put back afterwards.  The
        // levels below are the cycle's scratch (rs, Rs, vs, Vs of cpu-raw.lua:155-171), as in the reference.
        const int64_t n = level_count(Lv);
        const size_t bytes = (size_t)Lv.alloc * c->rb;
        TRY(materialize_zero(c, Lv));
        char *su = nullptr, *sf = nullptr;
        if (hipMalloc(&su, bytes) != hipSuccess || hipMalloc(&sf, bytes) != hipSuccess) {
            if (su) (void)hipFree(su);
            return c->fail(MGP_ERR_OOM, "mgp_two_grid: no room to save level %d", l);
        }
        int rc = MGP_OK;
        auto step = [&](int r) { if (rc == MGP_OK) rc = r; };
        step(hipMemcpyAsync(su, Lv.u, bytes, hipMemcpyDeviceToDevice, c->s) == hipSuccess ? MGP_OK : MGP_ERR_HIP);
        step(hipMemcpyAsync(sf, Lv.f, bytes, hipMemcpyDeviceToDevice, c->s) == hipSuccess ? MGP_OK : MGP_ERR_HIP);
        step(mgp_set_field(c, l, MGP_FIELD_U, u, n, mem));
        step(mgp_set_field(c, l, MGP_FIELD_F, f, n, mem));
        if (rc == MGP_OK && c->debug) {  // the reference checks inside twoGrid (cpu-raw.lua:126-140): a fresh record
            c->dbg_names.clear();
            step(hipMemsetAsync(c->d_dbg, 0x7f, sizeof(int), c->s) == hipSuccess ? MGP_OK : MGP_ERR_HIP);
        }
        if (rc == MGP_OK) step(cycle_rec(c, l, h, c->o.cycle == MGP_CYCLE_F));
        int dbg_first = -1;
        if (rc == MGP_OK && c->debug)
            step(hipMemcpy(&dbg_first, c->d_dbg, sizeof(int), hipMemcpyDeviceToHost) == hipSuccess ? MGP_OK : MGP_ERR_HIP);
        if (rc == MGP_OK && dbg_first >= 0 && dbg_first < (int)c->dbg_names.size())
            rc = c->fail(MGP_ERR_STATE, "found a nan (cpu-raw.lua:135-139, gpu.lua:279-283): %s",
                         c->dbg_names[(size_t)dbg_first].c_str());
        if (c->debug) c->dbg_names.clear();
        step(mgp_get_field(c, l, MGP_FIELD_U, u, n, mem));
        TRY(materialize_zero(c, Lv));
        const bool r1 = hipMemcpyAsync(Lv.u, su, bytes, hipMemcpyDeviceToDevice, c->s) == hipSuccess;
        const bool r2 = hipMemcpyAsync(Lv.f, sf, bytes, hipMemcpyDeviceToDevice, c->s) == hipSuccess;
        const bool r3 = hipStreamSynchronize(c->s) == hipSuccess;
        (void)hipFree(su);
        (void)hipFree(sf);
        Lv.ghost_ok = Lv.fghost_ok = true;
        Lv.ghost_zero = false;
        if (rc != MGP_OK) return rc;
        if (!(r1 && r2 && r3)) return c->fail(MGP_ERR_HIP, "mgp_two_grid: restoring level %d failed", l);
        return MGP_OK;
    }
    return c->fail(MGP_ERR_ARG, "mgp_two_grid: no level of size %lld", (long long)L);
}


int mgp_smooth(mgp_ctx* c, int level, int sweeps)
{
    if (!c || check_level(c, level) != MGP_OK || sweeps < 0) return MGP_ERR_ARG;
    TRY(smooth(c, level, sweeps, level_h(c, level)));
    return sync_and_check(c);
}

int mgp_residual_restrict(mgp_ctx* c, int level)
{
    if (!c || level < 0 || level + 1 >= (int)c->lev.size()) return MGP_ERR_ARG;
    TRY(residual_restrict(c, level, level_h(c, level)));
    return sync_and_check(c);
}

int mgp_prolong_correct(mgp_ctx* c, int level)
{
    if (!c || level < 0 || level + 1 >= (int)c->lev.size()) return MGP_ERR_ARG;
    TRY(prolong_correct(c, level));
    return sync_and_check(c);
}

int mgp_coarse_solve(mgp_ctx* c)
{
    if (!c) return MGP_ERR_ARG;
    const int l = (int)c->lev.size() - 1;
    TRY(coarse_solve_at(c, l, level_h(c, l)));
    return sync_and_check(c);
}

int mgp_sync(mgp_ctx* c) { return c ? sync_and_check(c) : MGP_ERR_ARG; }

static int level_of_size(const mgp_ctx* c, int64_t size)
{
    for (int l = 1; l < (int)c->lev.size(); ++l)
        if (c->lev[l].p.nx == size) return l;
    return -1;
}

int mgp_set_coarse_level(mgp_ctx* c, int64_t size)
{
    if (!c) return MGP_ERR_ARG;
    TRY(sync_and_check(c));
    drop_graphs(c);
    if (size == 0) {
        c->tail_level = -1;
        return ensure_rscratch(c, true);  // the former tail levels now restrict per piece
    }
    const int l = level_of_size(c, size);
    if (l < 0) return c->fail(MGP_ERR_ARG, "mgp_set_coarse_level: no level >= 1 with nx = %lld", (long long)size);
    if (c->rk == mgp::kRealF32D)
        return c->fail(MGP_ERR_ARG, "mgp_set_coarse_level: the coarse engine evaluates in the real type; arith = "
                                    "MGP_ARITH_DOUBLE runs every level per piece");
    const int prev = c->tail_level;
    if (!try_tail(c, l)) {
        c->tail_level = prev;
        return c->fail(MGP_ERR_ARG, "mgp_set_coarse_level: levels from nx = %lld do not fit the one-workgroup coarse engine",
                       (long long)size);
    }
    return ensure_rscratch(c, true);
}

int mgp_set_coarse_handoff(mgp_ctx* c, int64_t size, mgp_coarse_fn fn, void* user)
{
    if (!c) return MGP_ERR_ARG;
    TRY(sync_and_check(c));
    drop_graphs(c);
    if (!fn) {
        c->handoff_level = -1;
        c->handoff_fn = nullptr;
        c->handoff_user = nullptr;
        plan_tail(c);
        return ensure_rscratch(c, true);
    }
    const int l = level_of_size(c, size);
    if (l < 0 || c->lev[l].p.dist)
        return c->fail(MGP_ERR_ARG, "mgp_set_coarse_handoff: no replicated level >= 1 with nx = %lld", (long long)size);
    c->handoff_level = l;
    c->handoff_fn = fn;
    c->handoff_user = user;
    if (c->tail_level >= 0 && c->tail_level <= l) c->tail_level = -1;  // the levels below l are the callback's
    return ensure_rscratch(c, true);
}

int mgp_metrics(mgp_ctx* c, double* rel_err, int64_t* count, double* frob)
{
    if (!c) return MGP_ERR_ARG;
    if (!c->metrics_old)
        return c->fail(MGP_ERR_STATE, "mgp_metrics: no psiOld of a last outer iteration (run mgp_cycle with err_mode 1; "
                                      "not kept with MGP_KEEP_PSI_OLD=0 on the temporally blocked finest level)");
    if (!c->d_metrics) HIP_TRY(c, hipMalloc(&c->d_metrics, sizeof(double) * (3 * mgp::kSumBlocks + 3)));
    const Level& L0 = c->lev[0];
    double* out = c->d_metrics + 3 * mgp::kSumBlocks;
    HIP_TRY(c, mgp::launch_metrics(c->rb, c->ui(L0, L0.u), c->metrics_old, L0.g.P * L0.g.nz, c->d_metrics, out, c->s));
    WaitScope w(c);  // the all-reduce and the read-back after it wait for the peers
    if (c->multi()) {
        if (c->lb)
            TRY(lb_allreduce(c, out, 3));
        else
            NCCL_CALL(c, c->comm, ncclAllReduce(out, out, 3, ncclDouble, ncclSum, c->comm, c->s), "metrics all-reduce");
    }
    double h[3];
    HIP_TRY(c, hipMemcpyAsync(h, out, sizeof h, hipMemcpyDeviceToHost, c->s));
    TRY(sync_and_check(c));
    const int64_t n = (int64_t)h[1];
    if (rel_err) *rel_err = n > 0 ? h[0] / (double)n : NAN;    // test-gpu-obj.lua:240-243
    if (count) *count = n;
    if (frob) *frob = std::sqrt(h[2] / (double)c->ncells_global());  // gpu.lua:361-366
    return MGP_OK;
}

int mgp_residual_norm(mgp_ctx* c, int level, double* rnorm, double* fnorm)
{
    if (!c) return MGP_ERR_ARG;
    if (check_level(c, level) != MGP_OK) return c->fail(MGP_ERR_ARG, "mgp_residual_norm: bad level %d", level);
    Level& L = c->lev[level];
    TRY(materialize_zero(c, L));
    TRY(exchange(c, L));
    const int nb = mgp::resnorm_blocks(c->rk, L.g);
    const int64_t need = 2 * (int64_t)(nb + mgp::sum_scratch(nb)) + 2;
    if (need > c->d_rn_cap) {
        if (c->d_rn) HIP_TRY(c, hipFree(c->d_rn));
        c->d_rn = nullptr;
        c->d_rn_cap = 0;
        HIP_TRY(c, hipMalloc(&c->d_rn, sizeof(double) * need));
        c->d_rn_cap = need;
    }
    double* out = c->d_rn + need - 2;
    HIP_TRY(c, mgp::launch_residual_norm(c->rk, c->o.dim, c->ui(L, L.u), c->ui(L, L.f), L.g, level_h(c, level),
                                         coarse_coef(c->o.coarse_bc, level), c->d_rn, out, c->s));
    WaitScope w(c);  // the all-reduce and the read-back after it wait for the peers
    if (L.p.dist) {
        if (c->lb)
            TRY(lb_allreduce(c, out, 2));
        else
            NCCL_CALL(c, c->comm, ncclAllReduce(out, out, 2, ncclDouble, ncclSum, c->comm, c->s), "norm all-reduce");
    }
    double h[2];
    HIP_TRY(c, hipMemcpyAsync(h, out, sizeof h, hipMemcpyDeviceToHost, c->s));
    TRY(sync_and_check(c));
    if (rnorm) *rnorm = std::sqrt(h[0]);
    if (fnorm) *fnorm = std::sqrt(h[1]);
    return MGP_OK;
}

int mgp_cg_solve(mgp_ctx* c, double epsilon, int32_t maxiter, void* x_out, int mem, int32_t* iters, double* err,
                 double* linf_hist)
{
    if (!c || maxiter < 0) return MGP_ERR_ARG;
    if (c->o.world > 1) return c->fail(MGP_ERR_STATE, "mgp_cg_solve: single-GPU contexts only");
    Level& L = c->lev[0];
    const size_t bytes = (size_t)L.alloc * c->rb;
    std::vector<char*> buf(4, nullptr);
    double* scratch = nullptr;
    void* lex = nullptr;
    const int64_t count = level_count(L);
    auto release = [&] {
        for (char* b : buf)
            if (b) (void)hipFree(b);
        if (scratch) (void)hipFree(scratch);
        if (lex && lex != x_out) (void)hipFree(lex);
    };
    for (auto& b : buf)
        if (hipMalloc(&b, bytes) != hipSuccess || hipMemsetAsync(b, 0, bytes, c->s) != hipSuccess) {
            release();
            return c->fail(MGP_ERR_OOM, "mgp_cg_solve: no room for the CG vectors");
        }
    if (hipMalloc(&scratch, sizeof(double) * mgp::cg_scratch_doubles()) != hipSuccess) {
        release();
        return c->fail(MGP_ERR_OOM, "mgp_cg_solve: no room for the CG scratch");
    }
    mgp::CgArgs a{};
    a.g = L.g;
    a.h = level_h(c, 0);
    a.cl = 0.0;
    a.x = c->ui(L, buf[0]);
    a.r = c->ui(L, buf[1]);
    a.p = c->ui(L, buf[2]);
    a.q = c->ui(L, buf[3]);
    a.b = c->ui(L, L.f);
    a.scratch = scratch;
    a.x0_neg_b = true;  // converge-multigrid-vs-krylov.lua:45-46: x = -f, b = f
    a.maxiter = maxiter;
    a.epsilon = epsilon;
    a.linf = linf_hist;
    hipError_t e = mgp::launch_cg(c->rb, c->o.dim, a, c->s);
    if (e == hipSuccess && x_out) {
        if (mem == MGP_MEM_DEVICE) lex = x_out;
        else e = hipMalloc(&lex, (size_t)count * c->rb);
        if (e == hipSuccess) e = mgp::launch_unpack(c->rb, a.x, lex, L.g, c->s);
        if (e == hipSuccess && mem != MGP_MEM_DEVICE)
            e = hipMemcpyAsync(x_out, lex, (size_t)count * c->rb, hipMemcpyDeviceToHost, c->s);
        if (e == hipSuccess) e = hipStreamSynchronize(c->s);
    }
    release();
    if (e != hipSuccess) return c->fail(MGP_ERR_HIP, "mgp_cg_solve: %s", hipGetErrorString(e));
    if (iters) *iters = a.iters;
    if (err) *err = a.err;
    return MGP_OK;
}

int mgp_set_debug(mgp_ctx* c, int mode)
{
    if (!c || mode < 0 || mode > 1) return MGP_ERR_ARG;
    TRY(sync_and_check(c));
    if (mode && !c->d_dbg) HIP_TRY(c, hipMalloc(&c->d_dbg, sizeof(int)));
    c->debug = mode;
    return MGP_OK;
}

int mgp_timing(mgp_ctx* c, int enable)
{
    if (!c) return MGP_ERR_ARG;
    TRY(sync_and_check(c));
    if (enable && c->ev.empty()) {
        c->ev.resize(4096);
        c->ev_meta.resize(2048);
        for (auto& e : c->ev) HIP_TRY(c, hipEventCreate(&e));
    }
    c->timing = enable != 0;
    c->ev_used = 0;
    for (int k = 0; k < MGP_TIMING_KINDS; ++k) {
        c->t_ms[k] = 0.0;
        c->t_launch[k] = 0;
        c->t_bytes[k] = 0.0;
        c->t_info[k] = {};
    }
    return MGP_OK;
}

int mgp_timing_kernel(mgp_ctx* c, int kind, char* name, int cap, int64_t* grid)
{
    if (!c || kind < 0 || kind >= MGP_TIMING_KINDS || cap < 1 || !name) return MGP_ERR_ARG;
    const mgp::LaunchInfo& i = c->t_info[kind];
    std::snprintf(name, (size_t)cap, "%s", i.name);
    if (grid) *grid = i.grid;
    return i.name[0] ? MGP_OK : MGP_ERR_STATE;
}

int mgp_comm_log(mgp_ctx* c, int64_t* rows, int max_rows, int reset)
{
    if (!c || max_rows < 0 || (max_rows > 0 && !rows)) return MGP_ERR_ARG;
    const int n = (int)c->clog.size();
    for (int i = 0; i < n && i < max_rows; ++i) {
        const auto& r = c->clog[(size_t)i];
        int64_t* o = rows + 5 * i;
        o[0] = r.op;
        o[1] = r.side;
        o[2] = r.level;
        o[3] = r.msgs;
        o[4] = r.bytes;
    }
    if (reset) c->clog.clear();
    return n;
}

int mgp_timing_read(mgp_ctx* c, int kind, double* ms_total, int64_t* launches, double* bytes)
{
    if (!c || kind < 0 || kind >= MGP_TIMING_KINDS) return MGP_ERR_ARG;
    TRY(sync_and_check(c));
    timing_collect(c);
    if (ms_total) *ms_total = c->t_ms[kind];
    if (launches) *launches = c->t_launch[kind];
    if (bytes) *bytes = c->t_bytes[kind];
    return MGP_OK;
}

int mgp_copy_bandwidth(int device, int64_t bytes, int32_t reps, double* gbps)
{
    if (bytes < 16 || reps < 1 || !gbps) {
        g_create_error = "mgp_copy_bandwidth: bytes >= 16, reps >= 1 and an output are required";
        return MGP_ERR_ARG;
    }
    DeviceGuard keep_device;
    if (device >= 0 && hipSetDevice(device) != hipSuccess) {
        g_create_error = "mgp_copy_bandwidth: hipSetDevice failed";
        return MGP_ERR_HIP;
    }
    bytes &= ~(int64_t)15;
    void *a = nullptr, *b = nullptr;
    hipStream_t s = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    int rc = MGP_OK;
    double best = 0.0;
    if (hipMalloc(&a, (size_t)bytes) != hipSuccess || hipMalloc(&b, (size_t)bytes) != hipSuccess ||
        hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess || hipEventCreate(&e0) != hipSuccess ||
        hipEventCreate(&e1) != hipSuccess || hipMemsetAsync(a, 0, (size_t)bytes, s) != hipSuccess) {
        g_create_error = "mgp_copy_bandwidth: allocation failed";
        rc = MGP_ERR_OOM;
    }
    // every copy kernel shape, reps timed launches each after an untimed first touch; the best counts.
    // MGP_COPY_CALIB=1 adds the narrow-lane copies (FETCH_SIZE calibration, tools/fetch_calib.py).
    const char* calib = std::getenv("MGP_COPY_CALIB");
    const int kinds = calib && std::atoi(calib) ? mgp::kCopyCalibKinds : mgp::kCopyKinds;
    for (int kind = 0; kind < kinds && rc == MGP_OK; ++kind)
        for (int r = -1; r < reps && rc == MGP_OK; ++r) {
            if (hipEventRecord(e0, s) != hipSuccess || mgp::launch_copy16(kind, a, b, bytes, s) != hipSuccess ||
                hipEventRecord(e1, s) != hipSuccess || hipEventSynchronize(e1) != hipSuccess) {
                g_create_error = "mgp_copy_bandwidth: copy kernel failed";
                rc = MGP_ERR_HIP;
                break;
            }
            float ms = 0.f;
            (void)hipEventElapsedTime(&ms, e0, e1);
            if (r >= 0 && ms > 0.f) best = std::max(best, 2.0 * (double)bytes / (ms * 1e-3) / 1e9);
        }
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    if (s) (void)hipStreamDestroy(s);
    if (a) (void)hipFree(a);
    if (b) (void)hipFree(b);
    if (rc == MGP_OK) *gbps = best;
    return rc;
}

// =====================================================================================
// Single-process multi-GPU group (one Lua host driving the node's GPUs)
// =====================================================================================

struct mgp_group {
    std::vector<mgp_ctx*> ranks;
    std::vector<int> dev;
    mgp_loopback* lb = nullptr;  // all ranks on one device: loopback transport
    std::string err;
    std::atomic<bool> stop{false};  // a rank failed and the others were woken: the group is unusable
};


static thread_local std::string g_group_error;

// Wake the ranks still blocked on a failed rank: they would otherwise wait forever in a halo exchange or
// collective that rank never joined.  Loopback: break the host barrier.  RCCL: the group's communicators are
// non-blocking, so no rank thread sits inside an RCCL call for long (every call is polled to completion and
// the poll checks `stop`); once `stop` is set, no rank starts another call (NcclScope counts a call before
// it checks `stop`, so either the rank sees `stop` or this thread sees the call and waits for it), and when
// every rank's in-flight calls have returned, each communicator is aborted from here: its outstanding
// kernels exit, so a rank blocked in hipStreamSynchronize returns, sees `stop` and never touches it again.
static void group_abort(mgp_group* g)
{
    g->stop.store(true);
    if (g->lb) {
        std::lock_guard<std::mutex> lk(g->lb->m);
        g->lb->broken = true;
        g->lb->cv.notify_all();
        return;
    }
    for (auto* c : g->ranks)
        while (c && c->in_nccl.load() > 0) std::this_thread::yield();
    for (size_t r = 0; r < g->ranks.size(); ++r) {
        mgp_ctx* c = g->ranks[r];
        if (!c) continue;
        (void)hipSetDevice(g->dev[r]);
        if (c->xcomm) (void)ncclCommAbort(c->xcomm);
        if (c->comm) (void)ncclCommAbort(c->comm);
    }
}

// Run fn(rank context, r) on every rank, each in its own host thread with its device current (the
// ranks' halo exchanges and collectives must be issued concurrently).  First failure wins.  When a rank
// fails and the others have not returned within a short grace period, they are blocked on it: the group
// is aborted (group_abort) and unusable afterwards (every later call fails with MGP_ERR_STATE).
static int group_run(mgp_group* g, const std::function<int(mgp_ctx*, int)>& fn)
{
    if (g->stop.load()) {
        g->err = "group aborted after a rank failed: destroy it";
        return MGP_ERR_STATE;
    }
    DeviceGuard keep_device;
    const int n = (int)g->ranks.size();
    std::vector<int> rc((size_t)n, MGP_OK);
    std::mutex m;
    std::condition_variable cv;
    int done = 0;
    bool failed = false;
    int first = -1;  // the rank that failed first: the root cause (the others may fail because of it)
    // test hook: this rank fails at once, before any exchange (tests/test_gpu_group.py); read per call so that
    // a test can set it for one group only
    const char* fr = std::getenv("MGP_TEST_FAIL_RANK");
    const int fail_rank = fr ? std::atoi(fr) : -1;
    std::vector<std::thread> th;
    th.reserve((size_t)n);
    for (int r = 0; r < n; ++r)
        th.emplace_back([&, r] {
            int v;
            g->ranks[(size_t)r]->fail_after_sync = false;
            if (hipSetDevice(g->dev[(size_t)r]) != hipSuccess)
                v = MGP_ERR_HIP;
            else if (r == fail_rank)
                v = g->ranks[(size_t)r]->fail(MGP_ERR_STATE, "injected failure (MGP_TEST_FAIL_RANK)");
            else
                v = fn(g->ranks[(size_t)r], r);
            rc[(size_t)r] = v;
            std::lock_guard<std::mutex> lk(m);
            ++done;
            if (v != MGP_OK && !failed) {
                failed = true;
                first = r;
            }
            cv.notify_all();
        });
    bool aborted = false;
    {
        // after a failure, the others either finish (work that needs no peer) or block on the failed rank in an
        // exchange or collective (or in the stream synchronisation / read-back after one, all counted in
        // `waiting`): abort as soon as one of them waits, checked every 0.5 s, and in any case after
        // kAbortAfter (a peer-dependent wait the count misses must not hang the group)
        constexpr auto kAbortAfter = std::chrono::seconds(20);
        std::unique_lock<std::mutex> lk(m);
        cv.wait(lk, [&] { return done == n || failed; });
        const auto t_fail = std::chrono::steady_clock::now();
        while (done < n && !cv.wait_for(lk, std::chrono::milliseconds(500), [&] { return done == n; })) {
            bool blocked = std::chrono::steady_clock::now() - t_fail > kAbortAfter;
            for (int r = 0; r < n; ++r)
                blocked = blocked || (r != first && g->ranks[(size_t)r]->waiting.load() > 0);
            if (blocked) {
                lk.unlock();
                group_abort(g);
                aborted = true;
                break;
            }
        }
    }
    for (auto& t : th) t.join();
    // A rank failed and the others returned: their call sequences on the communicators no longer match (the
    // failed rank skipped what the others issued), so the group is unusable and its communicators are aborted
    // now (one rank included: ncclCommAbort then runs on the world-1 RCCL group).  Argument errors of every rank
    // alike, found before any peer call, leave the group usable, and so do failures raised only after a rank's
    // final synchronisation (the debug NaN check): every rank completed the call's collectives.
    if (first >= 0 && !aborted) {
        bool all_arg = true, late = true;
        for (int r = 0; r < n; ++r) {
            all_arg = all_arg && rc[(size_t)r] == MGP_ERR_ARG;
            late = late && (rc[(size_t)r] == MGP_OK || g->ranks[(size_t)r]->fail_after_sync);
        }
        if (!all_arg && !late) group_abort(g);
    }
    if (g->stop.load() && !g->lb)
        for (auto* c : g->ranks) c->comm = c->xcomm = nullptr;  // freed by ncclCommAbort
    if (first >= 0) {
        g->err = "rank " + std::to_string(first) + ": " + g->ranks[(size_t)first]->err;
        return rc[(size_t)first];
    }
    return MGP_OK;
}

void mgp_group_destroy(mgp_group* g)
{
    if (!g) return;
    DeviceGuard keep_device;
    for (auto* c : g->ranks)
        if (c) {
            (void)hipSetDevice(c->device);
            destroy_impl(c);
        }
    delete g->lb;
    delete g;
}

// The group's communicators: one rank per device, created by this one thread as NON-BLOCKING communicators
// (ncclConfig_t.blocking = 0; group_abort may then abort them from another thread), plus each rank's side-stream
// communicator.  Returns nullptr or an error message.
static const char* group_comms(const std::vector<int>& dev, std::vector<ncclComm_t>& comms, std::vector<ncclComm_t>& xcomms)
{
    static thread_local std::string msg;
    const int n = (int)dev.size();
    auto wait_all = [&](std::vector<ncclComm_t>& cs, const char* what) -> const char* {
        for (auto cm : cs) {
            ncclResult_t st = ncclInProgress;
            while (st == ncclInProgress)
                if (ncclCommGetAsyncError(cm, &st) != ncclSuccess) st = ncclInternalError;
            if (st != ncclSuccess) {
                msg = std::string(what) + ": " + ncclGetErrorString(st);
                return msg.c_str();
            }
        }
        return nullptr;
    };
    ncclUniqueId id;
    ncclResult_t r = ncclGetUniqueId(&id);
    if (r != ncclSuccess) {
        msg = std::string("ncclGetUniqueId: ") + ncclGetErrorString(r);
        return msg.c_str();
    }
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    r = ncclGroupStart();
    for (int q = 0; q < n && (r == ncclSuccess || r == ncclInProgress); ++q) {
        (void)hipSetDevice(dev[(size_t)q]);
        r = ncclCommInitRankConfig(&comms[(size_t)q], n, id, q, &cfg);
    }
    const ncclResult_t e = ncclGroupEnd();
    if (r == ncclSuccess) r = e;
    if (r != ncclSuccess && r != ncclInProgress) {
        msg = std::string("ncclCommInitRankConfig (non-blocking): ") + ncclGetErrorString(r);
        return msg.c_str();
    }
    if (const char* m = wait_all(comms, "communicator init")) return m;
    // the side-stream communicators: a second grouped non-blocking init with an id of their own (a grouped
    // ncclCommSplit of non-blocking communicators fails in RCCL 7.2 with "internal error": measured on the
    // one-device group, tests/test_gpu_rccl.py; the multi-process contexts split, one blocking call per rank)
    ncclUniqueId xid;
    r = ncclGetUniqueId(&xid);
    if (r != ncclSuccess) {
        msg = std::string("ncclGetUniqueId: ") + ncclGetErrorString(r);
        return msg.c_str();
    }
    r = ncclGroupStart();
    for (int q = 0; q < n && (r == ncclSuccess || r == ncclInProgress); ++q) {
        (void)hipSetDevice(dev[(size_t)q]);
        r = ncclCommInitRankConfig(&xcomms[(size_t)q], n, xid, q, &cfg);
    }
    const ncclResult_t e2 = ncclGroupEnd();
    if (r == ncclSuccess) r = e2;
    if (r != ncclSuccess && r != ncclInProgress) {
        msg = std::string("ncclCommInitRankConfig (side-stream communicators): ") + ncclGetErrorString(r);
        return msg.c_str();
    }
    return wait_all(xcomms, "side-stream communicator init");
}

int mgp_group_create(mgp_group** out, const mgp_opts* o, int ngpu, const int* devices)
{
    if (!out || !o || ngpu < 1) {
        g_create_error = "mgp_group_create: bad argument";
        return MGP_ERR_ARG;
    }
    *out = nullptr;
    DeviceGuard keep_device;
    mgp_group* g = new mgp_group();
    for (int r = 0; r < ngpu; ++r) g->dev.push_back(devices ? devices[r] : r);
    bool same = true;
    for (int d : g->dev) same = same && d == g->dev[0];
    mgp_opts ro = *o;
    ro.world = ngpu;
    ro.rank = 0;
    {
        std::vector<LevelPlan> plan;
        const int rc = plan_levels(ro, plan, g_create_error);
        if (rc != MGP_OK) {
            delete g;
            return rc;
        }
    }
    std::vector<ncclComm_t> comms((size_t)ngpu, nullptr), xcomms((size_t)ngpu, nullptr);
    if (ngpu > 1 && same) {
        mgp_loopback_create(&g->lb, ngpu);
    } else if (ngpu > 1 || env_rccl1(ro)) {  // (one device with MGP_TRANSPORT=rccl: a one-rank RCCL group)
        const char* rc_msg = group_comms(g->dev, comms, xcomms);
        if (rc_msg) {
            g_create_error = rc_msg;
            delete g;
            return MGP_ERR_RCCL;
        }
    }
    g->ranks.assign((size_t)ngpu, nullptr);
    for (int r = 0; r < ngpu; ++r) {
        ro.rank = r;
        ro.device = g->dev[(size_t)r];
        const int rc = create_impl(&g->ranks[(size_t)r], &ro, g->lb, comms[(size_t)r], xcomms[(size_t)r]);
        if (rc == MGP_OK) g->ranks[(size_t)r]->group_stop = &g->stop;
        if (rc != MGP_OK) {
            for (int q = r + 1; q < ngpu; ++q) {
                if (xcomms[(size_t)q]) (void)ncclCommDestroy(xcomms[(size_t)q]);
                if (comms[(size_t)q]) (void)ncclCommDestroy(comms[(size_t)q]);
            }
            const std::string e = g_create_error;
            mgp_group_destroy(g);
            g_create_error = "rank " + std::to_string(r) + ": " + e;
            return rc;
        }
    }
    *out = g;
    return MGP_OK;
}

int mgp_group_size(const mgp_group* g) { return g ? (int)g->ranks.size() : MGP_ERR_ARG; }

mgp_ctx* mgp_group_rank(mgp_group* g, int rank)
{
    return (g && rank >= 0 && rank < (int)g->ranks.size()) ? g->ranks[(size_t)rank] : nullptr;
}

const char* mgp_group_last_error(const mgp_group* g) { return g ? g->err.c_str() : g_create_error.c_str(); }

int mgp_group_init_point_charge(mgp_group* g)
{
    if (!g) return MGP_ERR_ARG;
    return group_run(g, [](mgp_ctx* c, int) { return mgp_init_point_charge(c); });
}

int mgp_group_cycles(mgp_group* g, int32_t k, double* errs)
{
    if (!g || k < 0) return MGP_ERR_ARG;
    return group_run(g, [&](mgp_ctx* c, int r) { return mgp_cycles(c, k, r == 0 && errs ? errs : nullptr); });
}

int mgp_group_cycle(mgp_group* g, double* err_out)
{
    double e = NAN;
    const int rc = mgp_group_cycles(g, 1, &e);
    if (err_out) *err_out = e;
    return rc;
}

// Global field of a level (x fastest, the whole box): each rank moves its own slab planes of a
// distributed level; a replicated level is read from rank 0 and written to every rank.
static int group_field_io(mgp_group* g, int level, int which, void* buf, int64_t count, int mem, bool to_device)
{
    if (!g || !buf) return MGP_ERR_ARG;
    mgp_ctx* c0 = g->ranks[0];
    if (check_level(c0, level) != MGP_OK) {
        g->err = "bad level";
        return MGP_ERR_ARG;
    }
    const LevelPlan& p = c0->lev[(size_t)level].p;
    const int64_t plane = p.nx * p.ny;
    if (count != plane * p.gnz) {
        g->err = "count " + std::to_string(count) + " != " + std::to_string(plane * p.gnz);
        return MGP_ERR_ARG;
    }
    return group_run(g, [&](mgp_ctx* c, int r) -> int {
        const Level& L = c->lev[(size_t)level];
        if (!L.p.dist && r > 0 && !to_device) return MGP_OK;
        char* at = (char*)buf + (size_t)(L.p.z0 * plane) * c->rb;
        return planes_io(c, level, which, 0, L.g.nz, at, mem, to_device);
    });
}

int mgp_group_get_field(mgp_group* g, int level, int which, void* dst, int64_t count, int mem)
{
    return group_field_io(g, level, which, dst, count, mem, false);
}

int mgp_group_set_field(mgp_group* g, int level, int which, const void* src, int64_t count, int mem)
{
    return group_field_io(g, level, which, const_cast<void*>(src), count, mem, true);
}

int mgp_group_residual_norm(mgp_group* g, int level, double* rnorm, double* fnorm)
{
    if (!g) return MGP_ERR_ARG;
    std::vector<double> rn(g->ranks.size()), fn(g->ranks.size());
    TRY(group_run(g, [&](mgp_ctx* c, int r) { return mgp_residual_norm(c, level, &rn[(size_t)r], &fn[(size_t)r]); }));
    if (rnorm) *rnorm = rn[0];  // all-reduced: every rank holds the global norms
    if (fnorm) *fnorm = fn[0];
    return MGP_OK;
}

int mgp_group_field_stats(mgp_group* g, int level, int which, uint64_t* hash, double stats[3])
{
    if (!g) return MGP_ERR_ARG;
    const size_t n = g->ranks.size();
    std::vector<uint64_t> h(n);
    std::vector<double> d(3 * n);
    TRY(group_run(g, [&](mgp_ctx* c, int r) { return mgp_field_stats(c, level, which, &h[(size_t)r], &d[3 * (size_t)r]); }));
    const bool dist = g->ranks[0]->lev[(size_t)level].p.dist;
    uint64_t hh = 0;
    double s = 0, q = 0, mx = 0;
    for (size_t r = 0; r < (dist ? n : 1); ++r) {
        hh += h[r];
        s += d[3 * r];
        q += d[3 * r + 1];
        mx = std::max(mx, d[3 * r + 2]);
    }
    if (hash) *hash = hh;
    if (stats) {
        stats[0] = s;
        stats[1] = q;
        stats[2] = mx;
    }
    return MGP_OK;
}

}  // extern "C"
