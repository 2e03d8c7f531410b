// pss_runtime.cpp -- native runtime behind include/pss.h.
//
// Owns a sampler handle: the reference's constructor math (V1:16-56), its stateful epoch
// history (init_iter, V1:100-132 / V2:124-159) evaluated on the host with a CPython-exact
// MT19937, the device buffers of the current epoch, and the kernel launches.
#include <hip/hip_runtime.h>
#include <sched.h>

#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/pss.h"
#include "pss_common.h"
#include "pss_kernels.h"
#include "pss_host_mt.h"
#include "pss_cpu.h"
#include "pss_map.h"

using pss::CPythonMT;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}

#define PSS_HIP(call)                                                                     \
    do {                                                                                  \
        hipError_t e_ = (call);                                                           \
        if (e_ != hipSuccess)                                                             \
            return fail(e_ == hipErrorNotSupported ? PSS_ENOTSUP : PSS_EHIP,              \
                        std::string(#call) + ": " + hipGetErrorString(e_));               \
    } while (0)

// The file-order permutation of an epoch (V1:114-117 seed(e + 1), V2:143-144 seed(e)):
// MT19937 Fisher-Yates of range(F).  A pure function of (version, epoch, F), so it can be
// computed ahead of time: the sampler prefetches the coming epochs' permutations on worker
// threads while the current epoch runs (init_iter then only composes it with the current
// order), and the O(F) host shuffle leaves the epoch's critical path.  One permutation costs
// ~16-25 ns per file, so at F = 80K (8 GPUs of C2 files) it is 1.3-2 ms against a ~0.2 ms
// epoch on the GPU: the prefetch depth, and the worker count, grow with F (one epoch ahead per
// 4096 files, 2..16, at most half the CPUs of the process's affinity mask).  Consumed
// permutation buffers are recycled to the workers (no per-epoch 320 KB mmap / munmap).
std::shared_ptr<std::vector<int32_t>> file_permutation(int32_t version, int64_t epoch, int64_t F,
                                                       std::shared_ptr<std::vector<int32_t>> v = nullptr) {
    if (!v) v = std::make_shared<std::vector<int32_t>>();
    v->resize(F);
    for (int64_t i = 0; i < F; i++) (*v)[i] = (int32_t)i;
    CPythonMT mt;
    mt.seed(version == 1 ? epoch + 1 : epoch);
    mt.shuffle(v->data(), F);
    return v;
}

class PermPrefetcher {
  public:
    PermPrefetcher(int32_t version, int64_t F) : version_(version), F_(F) {
        int64_t a = F / 4096;
        // the CPUs this process may run on (one process per GPU shares the node)
        int64_t hw = (int64_t)std::thread::hardware_concurrency();
        cpu_set_t set;
        CPU_ZERO(&set);
        if (sched_getaffinity(0, sizeof(set), &set) == 0 && CPU_COUNT(&set) > 0) hw = CPU_COUNT(&set);
        const int64_t cap = hw >= 4 ? hw / 2 : 2;
        a = a < 2 ? 2 : (a > 16 ? 16 : a);
        ahead_ = a < cap ? a : (cap < 2 ? 2 : cap);
    }
    ~PermPrefetcher() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto &t : workers_) t.join();
    }
    // the permutation of `epoch`: from the cache, or computed here (waiting for a worker that
    // is already on it); afterwards epochs epoch+1, epoch+2 are queued for the workers
    std::shared_ptr<std::vector<int32_t>> take(int64_t epoch) {
        std::shared_ptr<std::vector<int32_t>> r;
        {
            std::unique_lock<std::mutex> lk(mu_);
            cv_.wait(lk, [&] { return !busy_.count(epoch); });
            auto it = done_.find(epoch);
            if (it != done_.end()) { r = it->second; done_.erase(it); }
            // drop stale entries (epochs behind the caller, or far ahead)
            for (auto j = done_.begin(); j != done_.end();)
                j = (j->first < epoch || j->first > epoch + ahead_) ? done_.erase(j) : std::next(j);
        }
        if (!r) r = file_permutation(version_, epoch, F_, spare());
        for (int64_t d = 1; d <= ahead_; d++) request(epoch + d);
        return r;
    }
    // a consumed permutation's buffer back to the workers: no per-epoch allocation (a 320 KB
    // vector is an mmap, and its free an munmap with a TLB shootdown across the workers)
    void recycle(std::shared_ptr<std::vector<int32_t>> v) {
        if (!v || v.use_count() != 1) return;
        std::lock_guard<std::mutex> lk(mu_);
        if (free_.size() < (size_t)ahead_ + 2) free_.push_back(std::move(v));
    }

  private:
    int64_t ahead_ = 2;
    int32_t version_;
    int64_t F_;
    std::mutex mu_;
    std::condition_variable cv_;
    std::map<int64_t, std::shared_ptr<std::vector<int32_t>>> done_;
    std::map<int64_t, bool> busy_;
    std::vector<int64_t> queue_;
    std::vector<std::thread> workers_;
    std::vector<std::shared_ptr<std::vector<int32_t>>> free_;
    bool stop_ = false;

    std::shared_ptr<std::vector<int32_t>> spare() {
        std::lock_guard<std::mutex> lk(mu_);
        if (free_.empty()) return nullptr;
        auto v = std::move(free_.back());
        free_.pop_back();
        return v;
    }

    void request(int64_t e) {
        {
            std::lock_guard<std::mutex> lk(mu_);
            if (done_.count(e) || busy_.count(e)) return;
            for (int64_t q : queue_) if (q == e) return;
            queue_.push_back(e);
            if (workers_.size() < (size_t)ahead_) workers_.emplace_back([this] { run(); });
        }
        cv_.notify_all();
    }
    void run() {
        std::unique_lock<std::mutex> lk(mu_);
        for (;;) {
            cv_.wait(lk, [&] { return stop_ || !queue_.empty(); });
            if (stop_) return;
            const int64_t e = queue_.front();
            queue_.erase(queue_.begin());
            busy_[e] = true;
            std::shared_ptr<std::vector<int32_t>> buf;
            if (!free_.empty()) { buf = std::move(free_.back()); free_.pop_back(); }
            lk.unlock();
            auto v = file_permutation(version_, e, F_, std::move(buf));
            lk.lock();
            busy_.erase(e);
            done_[e] = v;
            cv_.notify_all();
        }
    }
};

class DeviceGuard {  // run on the handle's device, restore the caller's afterwards
  public:
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev_) != hipSuccess) prev_ = -1;
        if (prev_ != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        int cur = -1;
        if (prev_ >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev_) (void)hipSetDevice(prev_);
    }

  private:
    int prev_ = -1;
};

template <typename T>
struct DevBuf {
    T *p = nullptr;
    size_t n = 0;  // elements
    hipError_t ensure(size_t want) {
        if (want <= n && p) return hipSuccess;
        if (p) { (void)hipFree(p); p = nullptr; n = 0; }
        hipError_t e = hipMalloc((void **)&p, (want ? want : 1) * sizeof(T));
        if (e == hipSuccess) n = want;
        return e;
    }
    void release() { if (p) (void)hipFree(p); p = nullptr; n = 0; }
};

// Pinned host staging that k_upload reads (the per-epoch tables, a large rank table), as a ring
// of kN buffers: the host rewrites a buffer only after the upload that read it, and with a ring
// that upload is kN - 1 calls back.  (Round 6: with two table sets the host waited on the
// previous set's upload event every epoch -- hipEventSynchronize returned only as the NEXT
// upload on the table stream finished, ~110 us into the running replay -- so the host, not the
// GPU, paced the C2 mapped loop: 31 us between replays against 10 for the id loop.)
struct StageRing {
    static constexpr int kN = 4;
    void *buf[kN] = {};
    hipEvent_t ev[kN] = {};
    bool used[kN] = {};
    int next = 0;
    hipError_t init(size_t bytes) {
        for (int i = 0; i < kN; i++) {
            hipError_t e = hipHostMalloc(&buf[i], bytes ? bytes : 16);
            if (e == hipSuccess) e = hipEventCreateWithFlags(&ev[i], hipEventDisableTiming);
            if (e != hipSuccess) return e;
        }
        return hipSuccess;
    }
    hipError_t acquire(void **p, int *slot) {
        const int i = next;
        next = (next + 1) % kN;
        if (used[i]) {
            const hipError_t e = hipEventSynchronize(ev[i]);
            if (e != hipSuccess) return e;
        }
        *p = buf[i];
        *slot = i;
        return hipSuccess;
    }
    hipError_t release(int slot, hipStream_t s) {   // after the upload that reads it
        used[slot] = true;
        return hipEventRecord(ev[slot], s);
    }
    void destroy() {
        for (int i = 0; i < kN; i++) {
            if (ev[i]) {
                if (used[i]) (void)hipEventSynchronize(ev[i]);
                (void)hipEventDestroy(ev[i]);
            }
            if (buf[i]) (void)hipHostFree(buf[i]);
            ev[i] = nullptr;
            buf[i] = nullptr;
            used[i] = false;
        }
    }
};

}  // namespace

struct pss_sampler {
    // constructor state (V1:27-56)
    std::vector<int64_t> files_len;
    int64_t F = 0, N = 0, ns = 0, B = 0;
    int32_t R = 0, version = 1, shuffle = 1, device = 0;
    bool cpu = false;             // PSS_DEVICE_CPU: host threads, host pointers, no HIP call
    std::vector<int64_t> h_prefix;   // CPU mode: prefix over the epoch's file order
    double cpu_ms[pss::K_NUM_KINDS] = {};
    int64_t cpu_calls[pss::K_NUM_KINDS] = {};
    int32_t emit_path = 0;        // pss::EmitPath
    int32_t order_mode = 0;       // PSS_ORDER_COUNTER / PSS_ORDER_EXACT
    std::unique_ptr<PermPrefetcher> perms;   // file permutations of the coming epochs
    uint64_t seed = 0;
    // history state
    std::vector<int32_t> order;   // self.files as dataset positions
    std::vector<int32_t> order_next;   // init_iter's composition buffer (kept: no per-epoch allocation)
    std::vector<int32_t> blocks;  // self.blocks
    std::vector<pss::RankDesc> ranks;
    int64_t epoch = 0;
    bool iterated = false;
    // device state
    bool dev_init = false;
    bool dirty = true;            // rank descriptors of the epoch not on the device yet
    bool prefix_dirty = true;     // CPU mode: the host prefix is owed (cpu_prefix)
    DevBuf<int64_t> d_lens, d_ids;   // d_ids: scratch ids of pss_generate_mapped
    // The epoch's device tables -- the file order, its exclusive prefix and the prefix's bucket
    // index (pss_map.h; kb / nb below) -- in two sets.  A set is computed on the host on first use
    // after an init_iter (tables_host: O(F + nb), the host runs ahead of the GPU) into pinned
    // staging and uploaded as one blob by a short copy kernel on the handle's table stream, beside
    // epoch e - 1's kernels; the caller's stream only waits for it.  (Round 6: the device scan in
    // line cost ~30 us per epoch before a mapped replay at C2; the same three scan kernels on the
    // side stream delayed the replay's one round of waves by ~22 us, a one-workgroup scan by ~40.)
    // A set is rewritten after its last reader (`freed`); the staging comes from a ring (below).
    struct TabSet {
        DevBuf<uint32_t> blob;        // order | prefix | bucket index, 16-byte aligned parts
        int32_t *order = nullptr, *bucket = nullptr;
        int64_t *prefix = nullptr;
        hipEvent_t ready = nullptr, freed = nullptr;
        bool built = false, read = false;
    };
    StageRing tab_stage;          // pinned staging of the table blobs (the blob's layout)
    size_t tab_prefix_off = 0, tab_bucket_off = 0, tab_scratch_off = 0, tab_bytes = 0;   // blob layout (bytes)
    TabSet tab[2];
    int tab_cur = 0;
    bool tab_dirty = true;        // this epoch's tables not built yet
    hipStream_t tstream = nullptr;
    int32_t kb = 0;
    int64_t nb = 0, max_len = 0;
    pss::MapArgs map_sc{};        // host-known map shortcuts (map_shortcuts): T, pack, uni
    hipEvent_t ids_free = nullptr;   // last reader of d_ids
    DevBuf<int32_t> d_err;
    DevBuf<pss::RankDesc> d_ranks;
    DevBuf<uint32_t> d_val, d_buf, d_sort;
    StageRing rank_stage;         // pinned staging of the rank table (R > kArgRanksMax)
    // optional per-kernel timing (pss_profile): events recorded around every launch
    bool profiling = false;
    int32_t profile_mode = 0;     // 1 every launch, n >= 2 every (n-1)-th generation launch
    int64_t prof_seen = 0;        // generation launches seen in mode >= 2
    std::vector<hipEvent_t> ev_pool;
    size_t ev_used = 0;
    struct Span { int kind; size_t a, b; };
    std::vector<Span> spans;
    int open_kind = -1;
    size_t open_ev = 0;
    // V2 epoch lookahead: once generate() has been called with one shape for consecutive epochs,
    // the last-occurrence pass (VAL tables + key table, or the pools-beyond-LDS bucketing
    // workspace; all depend only on the epoch key and the shape) of epoch e+1 is queued on a low-priority side stream beside epoch e's replay, into the
    // other of two VAL buffers.  generate(e+1) with the same shape then launches the replay only.
    // PSS_V2_LOOKAHEAD=0 turns it off.
    static constexpr int kLaBufs = 3;   // VAL (and big-pool workspace) ring: d_val/d_buf + 2
    DevBuf<uint32_t> d_val2, d_buf2, d_val3, d_buf3;
    hipStream_t side = nullptr;
    hipEvent_t ev_side = nullptr;       // the last pass launched on the side stream
    hipEvent_t ev_pre = nullptr;        // the replay stream reached this call's mapped replay
    hipEvent_t ev_read[kLaBufs] = {};   // per buffer: the last replay that read it
    hipEvent_t ev_done[kLaBufs] = {};   // per buffer: the last lookahead pass that wrote it
    struct Shape {
        int64_t N, ns, B, pos_lo, count;
        int32_t R, rank_lo, nr, path;
        bool operator==(const Shape &o) const {
            return N == o.N && ns == o.ns && B == o.B && pos_lo == o.pos_lo && count == o.count &&
                   R == o.R && rank_lo == o.rank_lo && nr == o.nr && path == o.path;
        }
    };
    struct Pending { bool valid; Shape shape; uint32_t key0, key1; int buf; };
    Pending pend[2] = {};        // queued lookahead passes (epochs e+1, e+2)
    // Calls on different streams share the handle's device state (rank / order / prefix tables,
    // the V1 key table and exact-order workspace, the map scratch): a call that uses it first
    // waits for the last such call when that one ran on another stream (SharedUse).  The V2
    // counter-order replays of whole streams with their ranks as kernel arguments use none of it
    // (their VAL ring orders itself with events), so consecutive epochs on two streams overlap.
    // Exact-order draw lookahead: the reference's draws depend on the epoch and the windows alone
    // (V1:165-171; V2:107-109,147), so once pss_generate ran in exact order for consecutive
    // epochs of one call shape, the MT draws of the next epochs are made ahead into draw slots,
    // each on its own low-priority side stream (a few long windows keep ~11 CUs busy for
    // milliseconds: several epochs' draws run side by side).  The call of a prepared epoch only
    // decodes (V2) / resolves (V1).  PSS_EXACT_LOOKAHEAD=0 turns it off.
    static constexpr int kXSlots = 9;
    DevBuf<uint32_t> xslot[kXSlots];
    hipStream_t xside[kXSlots] = {};
    hipEvent_t xev_done[kXSlots] = {};   // per slot: its last draws
    hipEvent_t xev_read[kXSlots] = {};   // per slot: the last decode that read it
    struct XKey {                        // what a slot's draws depend on besides the epoch
        int32_t version;
        int64_t ns, B, pos_lo, pos_hi;   // (V2: the whole stream, positions 0, 0)
        bool operator==(const XKey &o) const {
            return version == o.version && ns == o.ns && B == o.B && pos_lo == o.pos_lo && pos_hi == o.pos_hi;
        }
    };
    struct XPend { bool valid; XKey key; int64_t epoch; };
    XPend xpend[kXSlots] = {};           // the epoch a slot holds (or is being filled with)
    // the last epoch called for each of a few recent call shapes (several rank or position
    // ranges per epoch each keep their own lookahead)
    struct XHist { bool valid; XKey key; int64_t epoch; uint64_t stamp; };
    static constexpr int kXHist = 4;
    XHist xhist[kXHist] = {};
    uint64_t xstamp = 0;
    // lookahead bounds (pss_set_lookahead): exact depth (-1: by geometry), the bytes all the draw
    // slots together may hold, V2 counter-order passes queued ahead (-1: 2); x_failed: an error
    // while preparing a slot turned the exact lookahead off for this handle (best effort)
    int32_t x_depth = -1, v2_depth = -1;
    int64_t x_cap = (int64_t)1 << 30;
    bool x_failed = false;
    int64_t st_x_made = 0, st_x_used = 0, st_v2_queued = 0, st_v2_used = 0;   // pss_lookahead_stats
    hipEvent_t ev_shared = nullptr;
    hipStream_t last_shared = nullptr;
    bool shared_used = false;
    bool last_valid = false;     // shape and epoch of the previous V2 generate
    Shape last_shape{};
    int64_t last_epoch = 0;

    pss::Geometry geometry() const {
        pss::Geometry g{};
        g.N = N; g.ns = ns; g.B = B; g.R = R; g.version = version;
        g.shuffle = version == 1 ? shuffle : 1;
        const uint64_t k = pss::epoch_key(seed, epoch);
        g.key0 = (uint32_t)k; g.key1 = (uint32_t)(k >> 32);
        return g;
    }
};

namespace {

// Marker callback: close the open span (if any) and open one for `kind` (kind < 0: close).
void prof_mark(void *ctx, int kind, hipStream_t s) {
    pss_sampler *h = (pss_sampler *)ctx;
    // mode n >= 2: generation kernels only, every (n - 1)-th launch; any other mark just closes
    // (nothing open: no event)
    if (h->profile_mode >= 2) {
        if (kind != pss::K_V1 && kind != pss::K_V2_EMIT) kind = -1;
        else if (h->prof_seen++ % (h->profile_mode - 1) != 0) kind = -1;
    }
    if (kind < 0 && h->open_kind < 0) return;
    if (h->ev_used == h->ev_pool.size()) {
        hipEvent_t e;
        if (hipEventCreate(&e) != hipSuccess) return;
        h->ev_pool.push_back(e);
    }
    const size_t e = h->ev_used++;
    (void)hipEventRecord(h->ev_pool[e], s);
    if (h->open_kind >= 0) h->spans.push_back({h->open_kind, h->open_ev, e});
    h->open_kind = kind;
    h->open_ev = e;
}

pss::Marker marker_of(pss_sampler *h) {
    pss::Marker m;
    if (h->profiling) { m.mark = prof_mark; m.ctx = h; }
    return m;
}

int ensure_device(pss_sampler *h) {
    if (h->dev_init) return PSS_OK;
    PSS_HIP(pss::init_kernel_attributes());
    PSS_HIP(h->d_lens.ensure((size_t)h->F));
    PSS_HIP(h->d_ranks.ensure((size_t)h->R));
    PSS_HIP(h->d_err.ensure(1));
    auto a16 = [](size_t b) { return (b + 15) & ~(size_t)15; };
    h->tab_prefix_off = a16(sizeof(int32_t) * (size_t)h->F);
    h->tab_bucket_off = a16(h->tab_prefix_off + sizeof(int64_t) * ((size_t)h->F + 1));
    h->tab_scratch_off = a16(h->tab_bucket_off + sizeof(int32_t) * (size_t)h->nb);
    h->tab_bytes = a16(h->tab_scratch_off + sizeof(uint64_t) * pss::scan_scratch_words(h->F));
    for (auto &t : h->tab) {
        PSS_HIP(t.blob.ensure(h->tab_bytes / sizeof(uint32_t)));
        char *b = (char *)t.blob.p;
        t.order = (int32_t *)b;
        t.prefix = (int64_t *)(b + h->tab_prefix_off);
        t.bucket = (int32_t *)(b + h->tab_bucket_off);
        PSS_HIP(hipEventCreateWithFlags(&t.ready, hipEventDisableTiming));
        PSS_HIP(hipEventCreateWithFlags(&t.freed, hipEventDisableTiming));
    }
    PSS_HIP(h->tab_stage.init(h->tab_bytes));
    PSS_HIP(hipStreamCreateWithFlags(&h->tstream, hipStreamNonBlocking));
    PSS_HIP(hipMemset(h->d_err.p, 0, sizeof(int32_t)));
    if (h->F) PSS_HIP(hipMemcpy(h->d_lens.p, h->files_len.data(), sizeof(int64_t) * h->F, hipMemcpyHostToDevice));
    PSS_HIP(h->rank_stage.init(sizeof(pss::RankDesc) * h->R));
    h->dev_init = true;
    return PSS_OK;
}

int prepare(pss_sampler *h, hipStream_t s) {
    if (!h->iterated) return fail(PSS_ESTATE, "pss_init_iter must be called before device work");
    int rc = ensure_device(h);
    if (rc) return rc;
    if (!h->dirty) return PSS_OK;
    // generation needs only the R rank descriptors: small tables travel as kernel arguments
    // (no copy-engine round trip on the epoch path), large ones through pinned staging
    if (h->R <= pss::kArgRanksMax) {
        PSS_HIP(pss::launch_put_ranks(h->ranks.data(), h->R, h->d_ranks.p, s));
    } else {
        int slot = 0;
        void *st = nullptr;
        PSS_HIP(h->rank_stage.acquire(&st, &slot));
        std::memcpy(st, h->ranks.data(), sizeof(pss::RankDesc) * h->R);
        PSS_HIP(pss::launch_upload(st, h->d_ranks.p, sizeof(pss::RankDesc) * h->R, s));
        PSS_HIP(h->rank_stage.release(slot, s));
    }
    h->dirty = false;
    return PSS_OK;
}

// The epoch's tables on the host (the device layout of a TabSet): the shuffled file order, its
// exclusive prefix over files_len (the reference's past_files_samples, V1:126,182-190; prefix[F] =
// the scanned total) and the bucket index BT[b] = file_of(prefix, F, b << kb) -- the largest f
// with prefix[f] <= b << kb: the non-empty file holding that id, F - 1 past the total (pss_map.h).
constexpr int64_t kHostTablesF = 16384;
void tables_host(const pss_sampler *h, int32_t *order, int64_t *prefix, int32_t *BT) {
    const int64_t F = h->F;
    std::memcpy(order, h->order.data(), sizeof(int32_t) * (size_t)F);
    int64_t run = 0, b = 0;
    for (int64_t f = 0; f < F; f++) {
        prefix[f] = run;
        const int64_t v = h->files_len[(size_t)order[f]];
        run += v;
        if (v > 0)
            for (; b < h->nb && (b << h->kb) < run; b++) BT[b] = (int32_t)f;
    }
    prefix[F] = run;
    for (; b < h->nb; b++) BT[b] = (int32_t)(F > 0 ? F - 1 : 0);
}

// The epoch's tables (TabSet: the shuffled file order, its prefix and bucket index), needed by
// the map, the fused hand-off, the gather and the partition only: built on first use after an
// init_iter into the other set, on the table stream, after that set's last reader; then `s`
// waits for them.  A call that reads them records tables_read on its stream afterwards.
int prepare_tables(pss_sampler *h, hipStream_t s) {
    if (!h->iterated) return fail(PSS_ESTATE, "pss_init_iter must be called before device work");
    int rc = ensure_device(h);
    if (rc) return rc;
#ifdef PSS_DIAG_TABLES_INLINE   // (timing-only build: the tables built in line on the caller's stream)
    h->tstream = s;
#endif
    if (h->tab_dirty) {
        const int k = h->tab_cur ^ 1;
        pss_sampler::TabSet &t = h->tab[k];
        int slot = 0;
        void *stv = nullptr;
        PSS_HIP(h->tab_stage.acquire(&stv, &slot));
        char *st = (char *)stv;
        // up to kHostTablesF files the host computes all three tables (O(F + nb), ~20 us at 10K
        // files, off the GPU); beyond, it stages the order only and the device scans it (at C3's
        // 100K files the host tables would sit on set_epoch -> first batch: 1.07 against 0.65 ms)
        const bool host = h->F <= kHostTablesF;
        if (host) tables_host(h, (int32_t *)st, (int64_t *)(st + h->tab_prefix_off), (int32_t *)(st + h->tab_bucket_off));
        else std::memcpy(st, h->order.data(), sizeof(int32_t) * (size_t)h->F);
        if (t.read) PSS_HIP(hipStreamWaitEvent(h->tstream, t.freed, 0));
        // Behind the last queued V2 lookahead pass too: that pass starts as the previous replay
        // ends, i.e. as this epoch's predecessor replay is launched, and the upload would otherwise
        // start right then and hold CU slots the one round of replay waves is waiting for (C2
        // mapped: replay 222 against 200 us).  After the pass it runs inside the replay instead.
        if (h->side && h->last_valid) PSS_HIP(hipStreamWaitEvent(h->tstream, h->ev_side, 0));
        const pss::Marker mk = marker_of(h);
        mk(pss::K_SCAN, h->tstream);
        if (host) {
            PSS_HIP(pss::launch_upload(st, t.blob.p, h->tab_scratch_off, h->tstream));   // order | prefix | index
        } else {
            PSS_HIP(pss::launch_upload(st, t.blob.p, sizeof(int32_t) * (size_t)h->F, h->tstream));
            PSS_HIP(pss::launch_scan_prefix(h->d_lens.p, t.order, h->F, t.prefix,
                                            (uint64_t *)((char *)t.blob.p + h->tab_scratch_off), h->tstream));
            PSS_HIP(pss::launch_bucket_index(t.prefix, h->F, h->kb, h->nb, t.bucket, h->tstream));
        }
        mk(-1, h->tstream);
        PSS_HIP(h->tab_stage.release(slot, h->tstream));
        PSS_HIP(hipEventRecord(t.ready, h->tstream));
        t.built = true;
        h->tab_cur = k;
        h->tab_dirty = false;
    }
    PSS_HIP(hipStreamWaitEvent(s, h->tab[h->tab_cur].ready, 0));
    return PSS_OK;
}

int tables_read(pss_sampler *h, hipStream_t s) {
    pss_sampler::TabSet &t = h->tab[h->tab_cur];
    PSS_HIP(hipEventRecord(t.freed, s));
    t.read = true;
    return PSS_OK;
}

// CPU mode: the exclusive prefix over the epoch's file order, computed on first use
int cpu_prefix(pss_sampler *h) {
    if (!h->iterated) return fail(PSS_ESTATE, "pss_init_iter must be called before generation");
    if (!h->prefix_dirty && (int64_t)h->h_prefix.size() == h->F + 1) return PSS_OK;
    h->h_prefix.resize((size_t)h->F + 1);
    pss::cpu::scan_prefix(h->files_len.data(), h->order.data(), h->F, h->h_prefix.data());
    h->prefix_dirty = false;
    return PSS_OK;
}

// RAII: device work on stream s that uses the handle's shared device state (see pss_sampler)
struct SharedUse {
    pss_sampler *h;
    hipStream_t s;
    SharedUse(pss_sampler *h_, hipStream_t s_) : h(h_), s(s_) {
        if (h->shared_used && h->last_shared != s && h->ev_shared)
            (void)hipStreamWaitEvent(s, h->ev_shared, 0);
    }
    ~SharedUse() {
#ifndef PSS_SHARED_EVENT_FLAGS
#define PSS_SHARED_EVENT_FLAGS hipEventDisableTiming
#endif
        if (!h->ev_shared && hipEventCreateWithFlags(&h->ev_shared, PSS_SHARED_EVENT_FLAGS) != hipSuccess) {
            h->ev_shared = nullptr;
            return;
        }
        if (hipEventRecord(h->ev_shared, s) == hipSuccess) {
            h->last_shared = s;
            h->shared_used = true;
        }
    }
};

struct CpuTimer {   // pss_profile in CPU mode: wall milliseconds per kernel kind
    pss_sampler *h;
    int kind;
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    ~CpuTimer() {
        if (!h->profiling) return;
        h->cpu_ms[kind] += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        h->cpu_calls[kind] += 1;
    }
};

// The map's host-known shortcuts (MapArgs: T, pack / pob, uni / uL / um / ul), fixed by the
// files' lengths at create -- the file order changes per epoch, the lengths and their total do not:
//   pack -- every pair (file position, offset) fits 31 bits as (file << pob) | offset, and every
//           virtual index fits 31 bits (an escaped slot value is kPairEsc | v): the exchange
//           replay carries pairs in its slot table (pss_device.h pair_window_consts)
//   uni  -- every file holds the same L > 0 samples and T < 2^32: the file position of id < T is
//           id / L (one multiply-high by a magic), offset id - file * L (prefix[f] = f * L in any
//           file order)
void map_shortcuts(pss_sampler *h, int64_t scanned) {
    pss::MapArgs &m = h->map_sc;
    m = pss::MapArgs{};
    m.T = scanned;
    const int64_t F = h->F;
    if (F <= 0 || h->max_len <= 0) return;
    uint32_t pob = 0;
    while (pob < 31 && (((int64_t)1 << pob) < h->max_len)) pob++;   // offsets < max_len <= 2^pob
    if (((F - 1) << pob) + (((int64_t)1 << pob) - 1) < ((int64_t)1 << 31) && h->ns < ((int64_t)1 << 31)) {
        m.pack = 1;
        m.pob = pob;
    }
    const int64_t L = h->files_len[0];
    bool uni = L > 0 && scanned < ((int64_t)1 << 32);
    for (int64_t i = 1; i < F && uni; i++) uni = h->files_len[i] == L;
    if (uni) {
        m.uni = 1;
        m.uL = (uint32_t)L;
        pss::udiv_magic((uint32_t)L, m.um, m.ul);
    }
}

// the map arguments of the current epoch's device tables and the caller's outputs
pss::MapArgs map_args(const pss_sampler *h, int32_t *fpos, int32_t *off) {
    pss::MapArgs m = h->map_sc;
    m.prefix = h->tab[h->tab_cur].prefix;
    m.F = h->F;
    m.BT = h->tab[h->tab_cur].bucket;
    m.kb = h->kb;
    m.nb = h->nb;
    m.fpos = fpos;
    m.off = off;
    return m;
}

}  // namespace

extern "C" {

const char *pss_last_error(void) { return g_err.c_str(); }
int pss_abi_version(void) { return 2; }

// counter-order schedule: 1 round 1, 2 round 2 (grouped pools, 24-bit slot hash), 3 round 3
// (16-bit round function at 10-bit halves, 8 fmix32 rounds at halves <= 5 bits), 4 round 6
// (grouped pools beyond 16384 slots: bursts of 32 steps per group instead of 16)
int pss_schedule_version(void) { return 4; }

int pss_create(const int64_t *files_len, int64_t num_files, int64_t total_size,
               int32_t num_replicas, int64_t shuffle_buffer, int32_t version, int32_t shuffle,
               uint64_t seed, int32_t device, pss_sampler **out) {
    if (!out) return fail(PSS_EINVAL, "out is NULL");
    *out = nullptr;
    if (num_files < 0 || (num_files > 0 && !files_len)) return fail(PSS_EINVAL, "bad files_len");
    if (num_files >= (int64_t)INT32_MAX) return fail(PSS_ENOTSUP, "more than 2^31-1 files");
    if (num_replicas <= 0) return fail(PSS_EINVAL, "num_replicas must be positive");
    if (shuffle_buffer <= 0) return fail(PSS_EINVAL, "shuffle_buffer must be positive");
    if (version != 1 && version != 2) return fail(PSS_EINVAL, "version must be 1 or 2");
    if (total_size <= 0) return fail(PSS_EINVAL, "total_size must be positive");
    pss_sampler *h = new pss_sampler();
    h->files_len.assign(files_len, files_len + num_files);
    int64_t scanned = 0;
    for (int64_t v : h->files_len) {
        if (v < 0) { delete h; return fail(PSS_EINVAL, "negative file length"); }
        scanned += v;
        if (v > h->max_len) h->max_len = v;
    }
    h->kb = pss::bucket_shift(scanned, num_files);
    h->nb = pss::bucket_count(scanned, h->kb);
    h->F = num_files;
    h->N = total_size;
    h->R = num_replicas;
    h->B = shuffle_buffer;
    h->version = version;
    h->shuffle = shuffle ? 1 : 0;
    h->seed = seed;
    h->device = device;
    h->cpu = device == PSS_DEVICE_CPU;
    h->ns = (int64_t)std::ceil((double)total_size / (double)num_replicas);  // V1:42 (float ceil)
    if (h->ns >= (int64_t)UINT32_MAX) { delete h; return fail(PSS_ENOTSUP, "num_samples >= 2^32 per rank"); }
    map_shortcuts(h, scanned);
    h->order.resize(num_files);
    for (int64_t i = 0; i < num_files; i++) h->order[i] = (int32_t)i;
    h->blocks.resize(num_replicas);
    for (int32_t r = 0; r < num_replicas; r++) h->blocks[r] = r;
    h->ranks.resize(num_replicas);
    for (int32_t r = 0; r < num_replicas; r++) {   // V1:52-53: start_num = ns * blocks[rank]
        h->ranks[r].old_start = h->ns * r;
        h->ranks[r].new_start = h->ns * r;
    }
    *out = h;
    return PSS_OK;
}

int pss_destroy(pss_sampler *h) {
    if (!h) return PSS_OK;
    if (h->dev_init && !h->cpu) {
        DeviceGuard dg(h->device);
        h->rank_stage.destroy();
        if (h->side) (void)hipStreamSynchronize(h->side);   // a lookahead still writing VAL
        if (h->tstream) (void)hipStreamSynchronize(h->tstream);
        (void)hipDeviceSynchronize();   // readers of the tables on the callers' streams
        h->d_lens.release(); h->d_err.release();
        h->d_ranks.release(); h->d_val.release(); h->d_buf.release(); h->d_sort.release();
        h->d_ids.release();
        for (auto &t : h->tab) {
            t.blob.release();
            for (hipEvent_t e : {t.ready, t.freed}) if (e) (void)hipEventDestroy(e);
        }
        if (h->tstream) (void)hipStreamDestroy(h->tstream);
        if (h->ids_free) (void)hipEventDestroy(h->ids_free);
        h->tab_stage.destroy();
        for (hipEvent_t e : h->ev_pool) (void)hipEventDestroy(e);
        if (h->side) (void)hipStreamDestroy(h->side);
        if (h->ev_side) (void)hipEventDestroy(h->ev_side);
        if (h->ev_pre) (void)hipEventDestroy(h->ev_pre);
        for (hipEvent_t e : h->ev_read) if (e) (void)hipEventDestroy(e);
        for (hipEvent_t e : h->ev_done) if (e) (void)hipEventDestroy(e);
        if (h->ev_shared) (void)hipEventDestroy(h->ev_shared);
        h->d_val2.release(); h->d_buf2.release(); h->d_val3.release(); h->d_buf3.release();
        for (int k = 0; k < pss_sampler::kXSlots; k++) {
            if (h->xside[k]) { (void)hipStreamSynchronize(h->xside[k]); (void)hipStreamDestroy(h->xside[k]); }
            if (h->xev_done[k]) (void)hipEventDestroy(h->xev_done[k]);
            if (h->xev_read[k]) (void)hipEventDestroy(h->xev_read[k]);
            h->xslot[k].release();
        }
    }
    delete h;
    return PSS_OK;
}

int pss_num_samples(const pss_sampler *h, int64_t *ns) {
    if (!h || !ns) return fail(PSS_EINVAL, "NULL argument");
    *ns = h->ns;
    return PSS_OK;
}

int pss_init_iter(pss_sampler *h, int64_t epoch) {
    if (!h) return fail(PSS_EINVAL, "NULL handle");
    CPythonMT mt;
    for (int32_t r = 0; r < h->R; r++) h->ranks[r].old_start = h->ranks[r].new_start;
    const bool files = h->version == 2 || h->shuffle;
    std::shared_ptr<std::vector<int32_t>> fid;
    if (files) {
        if (!h->perms) h->perms.reset(new PermPrefetcher(h->version, h->F));
        fid = h->perms->take(epoch);                    // V1:114-117 / V2:143-144
    }
    if (h->version == 1) {
        if (h->shuffle) {                              // V1:113-125
            mt.seed(epoch + 2);
            mt.shuffle(h->blocks.data(), h->R);        // cumulative: self.blocks is kept
        }
    } else {                                           // V2:142-152
        for (int32_t r = 0; r < h->R; r++) h->blocks[r] = r;
        mt.seed(epoch + 1);
        mt.shuffle(h->blocks.data(), h->R);
    }
    if (files) {                                       // cumulative: self.files is re-shuffled
        std::vector<int32_t> &o = h->order_next;
        o.resize(h->F);
        const int32_t *f = fid->data();
        for (int64_t i = 0; i < h->F; i++) o[i] = h->order[f[i]];
        h->order.swap(o);
        h->perms->recycle(std::move(fid));
    }
    for (int32_t r = 0; r < h->R; r++) h->ranks[r].new_start = h->ns * (int64_t)h->blocks[r];
    h->epoch = epoch;
    h->iterated = true;
    h->dirty = true;
    h->tab_dirty = true;
    h->prefix_dirty = true;
    return PSS_OK;
}

int pss_file_order(const pss_sampler *h, int32_t *order) {
    if (!h || (!order && h->F)) return fail(PSS_EINVAL, "NULL argument");
    std::memcpy(order, h->order.data(), sizeof(int32_t) * h->F);
    return PSS_OK;
}

int pss_blocks(const pss_sampler *h, int32_t *blocks) {
    if (!h || !blocks) return fail(PSS_EINVAL, "NULL argument");
    std::memcpy(blocks, h->blocks.data(), sizeof(int32_t) * h->R);
    return PSS_OK;
}

int pss_rank_starts(const pss_sampler *h, int64_t *old_start, int64_t *new_start) {
    if (!h) return fail(PSS_EINVAL, "NULL handle");
    for (int32_t r = 0; r < h->R; r++) {
        if (old_start) old_start[r] = h->ranks[r].old_start;
        if (new_start) new_start[r] = h->ranks[r].new_start;
    }
    return PSS_OK;
}

int pss_prepare(pss_sampler *h, void *stream) {
    if (!h) return fail(PSS_EINVAL, "NULL handle");
    if (h->cpu) return cpu_prefix(h);
    DeviceGuard dg(h->device);
    SharedUse su(h, (hipStream_t)stream);
    const int rc = prepare(h, (hipStream_t)stream);
    return rc ? rc : prepare_tables(h, (hipStream_t)stream);
}

namespace {

bool lookahead_on() {
    static const bool on = [] {
        const char *e = getenv("PSS_V2_LOOKAHEAD");
        return !(e && e[0] == '0');
    }();
    return on;
}

// V2 counter order, splittable shape: the replay of this epoch on `s`, its last-occurrence pass
// either taken from the lookahead queued by the previous call or run here; then, if the previous
// call had this shape at epoch - 1, the pass of epoch + 1 on the side stream.
int generate_v2_lookahead(pss_sampler *h, const pss::Geometry &g, int32_t rank_lo, int32_t nr,
                          int64_t pos_lo, int64_t count, int64_t *out_dev, hipStream_t s,
                          const pss::Marker &mk, const pss::MapArgs *ma, const pss::RankArgs *ra) {
    constexpr int NB = pss_sampler::kLaBufs;
    const size_t words = (pss::v2_val_bytes(g, nr) + sizeof(uint32_t) - 1) / sizeof(uint32_t);
    const size_t bwords = (pss::v2_buf_bytes(g, nr) + sizeof(uint32_t) - 1) / sizeof(uint32_t);
    DevBuf<uint32_t> *V[NB] = {&h->d_val, &h->d_val2, &h->d_val3};
    DevBuf<uint32_t> *W[NB] = {&h->d_buf, &h->d_buf2, &h->d_buf3};
    // buffers grow on first use: the one this call picks now, the other two only when a
    // lookahead pass is actually queued into them (one-off calls never triple the workspace)
    auto small = [&](int b) { return V[b]->n < words || (bwords && W[b]->n < bwords); };
    auto grow = [&](int b) -> int {
        if (!small(b)) return PSS_OK;
        if (h->side) PSS_HIP(hipStreamSynchronize(h->side));   // no pass may write a freed buffer
        // a queued pass of another shape into this buffer is dropped with it
        for (auto &p : h->pend) if (p.valid && p.buf == b) p.valid = false;
        PSS_HIP(hipDeviceSynchronize());    // its last reader (a replay on any stream) is done
        PSS_HIP(V[b]->ensure(words));
        if (bwords) PSS_HIP(W[b]->ensure(bwords));
        return PSS_OK;
    };
    if (!h->side) {
        int least = 0, greatest = 0;
        PSS_HIP(hipDeviceGetStreamPriorityRange(&least, &greatest));
        // the lowest priority: at the highest the C2 step was slower (519 vs 526 G idx/s, round 2)
        (void)greatest;
        PSS_HIP(hipStreamCreateWithPriority(&h->side, hipStreamNonBlocking, least));
        // these events only order device work on this device (never inspected by the host):
        // without the system-scope fence a step takes 176 against 179 us at C2, same box
        // (profiles/r04/ab_evflags; device-scope release alone: 179)
#ifndef PSS_LA_EVENT_FLAGS
#define PSS_LA_EVENT_FLAGS (hipEventDisableTiming | hipEventDisableSystemFence)
#endif
        for (hipEvent_t &e : h->ev_read) PSS_HIP(hipEventCreateWithFlags(&e, PSS_LA_EVENT_FLAGS));
        for (hipEvent_t &e : h->ev_done) PSS_HIP(hipEventCreateWithFlags(&e, PSS_LA_EVENT_FLAGS));
        PSS_HIP(hipEventCreateWithFlags(&h->ev_side, PSS_LA_EVENT_FLAGS));
        PSS_HIP(hipEventCreateWithFlags(&h->ev_pre, PSS_LA_EVENT_FLAGS));
    }
    // epochs queued ahead: 2 keeps the wait for a pass off the replay's critical path (one
    // epoch ahead: the replay waits 33 us per step, 491 against 526 G idx/s, round 2)
    const int depth = h->v2_depth < 0 ? 2 : h->v2_depth;   // (pss_set_lookahead; 0 never gets here)
    const pss_sampler::Shape shape{g.N, g.ns, g.B, pos_lo, count, g.R, rank_lo, nr, h->emit_path};
    auto held = [&](int b) {
        for (const auto &p : h->pend) if (p.valid && p.buf == b) return true;
        return false;
    };
    int buf = -1;
    bool pre = false;
    for (auto &p : h->pend)
        if (p.valid && p.shape == shape && p.key0 == g.key0 && p.key1 == g.key1) {
            buf = p.buf;
            p.valid = false;
        }
    if (buf >= 0 && small(buf)) buf = -1;   // (cannot happen: queued passes had their size)
    if (buf >= 0) {
        h->st_v2_used++;
#if !defined(PSS_DIAG_NO_STREAM_EVENTS) && !defined(PSS_DIAG_NO_STREAM_WAIT)
        // (diagnostics: the replay stream's gaps without its wait and/or record; racy)
        PSS_HIP(hipStreamWaitEvent(s, h->ev_done[buf], 0));
#endif
        // mapped: this call's passes wait until the replay stream reaches its replay.  The
        // mapped replay also waits for the epoch's tables (another stream), and the next pass,
        // released by the previous replay's end, would otherwise take the CUs first: the one
        // round of replay waves then starts ~25 us late (C2 mapped hand-off 0.260 -> 0.247 ms,
        // same box; the id replay, ahead of its pass already, loses ~2 % with the extra record)
        pre = ma != nullptr;
        if (pre) PSS_HIP(hipEventRecord(h->ev_pre, s));
        PSS_HIP(pss::launch_v2(g, h->d_ranks.p, rank_lo, nr, pos_lo, count, out_dev, V[buf]->p,
                               bwords ? W[buf]->p : nullptr, nullptr, h->d_err.p, s, mk, h->emit_path,
                               pss::V2_STAGE_EMIT, ma, ra));
    } else {
        // a buffer no queued lookahead holds, after its last reader and its last writer
        for (int b = 0; b < NB && buf < 0; b++) if (!held(b)) buf = b;
        { const int rc = grow(buf); if (rc) return rc; }
        PSS_HIP(hipStreamWaitEvent(s, h->ev_read[buf], 0));
        PSS_HIP(hipStreamWaitEvent(s, h->ev_done[buf], 0));
        PSS_HIP(pss::launch_v2(g, h->d_ranks.p, rank_lo, nr, pos_lo, count, out_dev, V[buf]->p,
                               bwords ? W[buf]->p : nullptr, nullptr, h->d_err.p, s, mk, h->emit_path,
                               pss::V2_STAGE_ALL, ma, ra));
    }
#if !defined(PSS_DIAG_NO_STREAM_EVENTS) && !defined(PSS_DIAG_NO_STREAM_RECORD)
    PSS_HIP(hipEventRecord(h->ev_read[buf], s));
#endif
    const bool sequential = h->last_valid && h->last_shape == shape && h->last_epoch == h->epoch - 1;
    h->last_valid = true;
    h->last_shape = shape;
    h->last_epoch = h->epoch;
    uint32_t k0[3], k1[3];
    for (int d = 1; d <= 2; d++) {
        const uint64_t k = pss::epoch_key(h->seed, h->epoch + d);
        k0[d] = (uint32_t)k; k1[d] = (uint32_t)(k >> 32);
    }
    for (auto &p : h->pend) {   // keep only passes of the coming epochs of this shape
        const bool next = p.valid && p.shape == shape &&
                          ((p.key0 == k0[1] && p.key1 == k1[1]) || (depth > 1 && p.key0 == k0[2] && p.key1 == k1[2]));
        if (!next || !sequential) p.valid = false;
    }
    if (!sequential) return PSS_OK;
    for (int d = 1; d <= depth; d++) {
        bool queued = false;
        for (const auto &p : h->pend) queued |= p.valid && p.key0 == k0[d] && p.key1 == k1[d];
        if (queued) continue;
        int nb = -1;
        for (int b = 0; b < NB && nb < 0; b++) if (b != buf && !held(b)) nb = b;
        if (nb < 0) break;
        { const int rc = grow(nb); if (rc) return rc; }
        pss::Geometry gn = g;
        gn.key0 = k0[d]; gn.key1 = k1[d];
        PSS_HIP(hipStreamWaitEvent(h->side, h->ev_read[nb], 0));   // the replay that read it
        if (pre) PSS_HIP(hipStreamWaitEvent(h->side, h->ev_pre, 0));
        PSS_HIP(pss::launch_v2(gn, h->d_ranks.p, rank_lo, nr, pos_lo, count, out_dev, V[nb]->p,
                               bwords ? W[nb]->p : nullptr, nullptr, h->d_err.p, h->side, mk, h->emit_path,
                               pss::V2_STAGE_PRE));
        PSS_HIP(hipEventRecord(h->ev_done[nb], h->side));
        PSS_HIP(hipEventRecord(h->ev_side, h->side));
        for (auto &p : h->pend)
            if (!p.valid) { p = {true, shape, k0[d], k1[d], nb}; break; }
        h->st_v2_queued++;
    }
    return PSS_OK;
}

bool exact_lookahead_on() {
    static const bool on = [] {
        const char *e = getenv("PSS_EXACT_LOOKAHEAD");
        return !(e && e[0] == '0');
    }();
    return on;
}

// Exact order: this epoch's decode (V2) / resolution (V1) from the draw slot a previous call
// prepared (else drawing first); then, if the previous call was epoch - 1 of this shape, the
// draws of the coming epochs into free slots on their side streams.
int generate_exact(pss_sampler *h, const pss::Geometry &g, int32_t rank_lo, int32_t nr, int64_t pos_lo,
                   int64_t count, int64_t *out_dev, hipStream_t s, const pss::Marker &mk) {
    constexpr int NX = pss_sampler::kXSlots;
    auto words = [](size_t bytes) { return (bytes + sizeof(uint32_t) - 1) / sizeof(uint32_t); };
    const int64_t e = h->epoch;
    const bool v1 = h->version == 1;
    const pss_sampler::XKey key{h->version, g.ns, g.B, v1 ? pos_lo : 0,
                                v1 ? (pos_lo + count < g.ns ? pos_lo + count : g.ns) : 0};
    int use = -1;
    for (int k = 0; k < NX; k++) {
        const auto &p = h->xpend[k];
        if (p.valid && p.key == key && p.epoch == e) use = k;
    }
    if (use >= 0) {
        PSS_HIP(hipStreamWaitEvent(s, h->xev_done[use], 0));
        h->xpend[use].valid = false;
        h->st_x_used++;
    }
    uint32_t *slot = use >= 0 ? h->xslot[use].p : nullptr;
    mk(v1 ? pss::K_V1 : pss::K_V2_EMIT, s);
    if (v1)
        PSS_HIP(pss::launch_v1_exact(g, h->d_ranks.p, rank_lo, nr, pos_lo, count, e, out_dev, h->d_sort.p, s,
                                     nullptr, slot));
    else
        PSS_HIP(pss::launch_v2_exact(g, h->d_ranks.p, rank_lo, nr, pos_lo, count, e, out_dev, h->d_sort.p, s,
                                     nullptr, slot));
    mk(-1, s);
    if (use >= 0) PSS_HIP(hipEventRecord(h->xev_read[use], s));
    // The lookahead below is best effort: this call's result is already enqueued, and nothing
    // that fails while preparing the coming epochs' slots fails the call -- the slot
    // is dropped, the exact lookahead turned off for the handle, PSS_OK returned.
    // (a later call of the same epoch and shape -- another rank range -- draws for itself: a slot
    // is used once, V2's decode takes K1 as scratch, V1's scan its bucket counts)
    int hx = -1;
    for (int i = 0; i < pss_sampler::kXHist; i++)
        if (h->xhist[i].valid && h->xhist[i].key == key) hx = i;
    if (hx >= 0 && h->xhist[hx].epoch == e) return PSS_OK;
    const bool sequential = hx >= 0 && h->xhist[hx].epoch == e - 1;
    if (hx < 0) {   // the least recently called shape's entry
        hx = 0;
        for (int i = 1; i < pss_sampler::kXHist; i++)
            if (!h->xhist[i].valid || (h->xhist[hx].valid && h->xhist[i].stamp < h->xhist[hx].stamp)) hx = i;
    }
    h->xhist[hx] = {true, key, e, ++h->xstamp};
    const size_t sbytes = v1 ? pss::v1_exact_slot_bytes(g, pos_lo, count) : pss::v2_exact_slot_bytes(g);
    const size_t sw = words(sbytes);
    int depth = (!exact_lookahead_on() || h->x_failed) ? 0
                : v1 ? pss::v1_exact_lookahead_depth(g, pos_lo, count) : pss::v2_exact_lookahead_depth(g);
    if (h->x_depth >= 0 && h->x_depth < depth) depth = h->x_depth;
    // the byte cap counts every slot that holds memory, the one this call's decode reads included
    const int64_t cap_slots = sbytes ? std::min<int64_t>(NX, h->x_cap / (int64_t)(sw * sizeof(uint32_t))) : 0;
    if (depth > cap_slots - 1) depth = (int)std::max<int64_t>(0, cap_slots - 1);
    for (auto &p : h->xpend) {   // keep the slots of the coming epochs of the shapes called lately
        if (!p.valid) continue;
        bool keep = false;
        for (const auto &x : h->xhist)
            keep |= x.valid && x.key == p.key && p.epoch > x.epoch && p.epoch <= x.epoch + depth;
        if (!keep) p.valid = false;
    }
    // memory of idle slots beyond what the bounds allow goes back (no host wait: slots still
    // being drawn or read are released by a later call)
    for (int k = 0; k < NX; k++) {
        if (!h->xslot[k].p || h->xpend[k].valid || k == use || (k < cap_slots && depth > 0)) continue;
        if (hipStreamQuery(h->xside[k]) == hipSuccess && hipEventQuery(h->xev_read[k]) == hipSuccess)
            h->xslot[k].release();
    }
    (void)hipGetLastError();   // (a query's hipErrorNotReady)
    if (!sequential || depth <= 0) return PSS_OK;
    auto prepare_slot = [&](int k, int64_t ep) -> hipError_t {
        hipError_t r;
        if (!h->xside[k]) {
            int least = 0, greatest = 0;
            if ((r = hipDeviceGetStreamPriorityRange(&least, &greatest)) != hipSuccess) return r;
            if ((r = hipStreamCreateWithPriority(&h->xside[k], hipStreamNonBlocking, least)) != hipSuccess) return r;
            if ((r = hipEventCreateWithFlags(&h->xev_done[k], PSS_LA_EVENT_FLAGS)) != hipSuccess) return r;
            if ((r = hipEventCreateWithFlags(&h->xev_read[k], PSS_LA_EVENT_FLAGS)) != hipSuccess) return r;
        }
        if (h->xslot[k].n < sw) {   // grows once: after its last draws and its last reader
            if ((r = hipStreamSynchronize(h->xside[k])) != hipSuccess) return r;
            if ((r = hipEventSynchronize(h->xev_read[k])) != hipSuccess) return r;
            if ((r = h->xslot[k].ensure(sw)) != hipSuccess) return r;
        }
        if ((r = hipStreamWaitEvent(h->xside[k], h->xev_read[k], 0)) != hipSuccess) return r;   // its last decode
        r = v1 ? pss::launch_v1_exact_draws(g, pos_lo, count, ep, h->xslot[k].p, h->xside[k])
               : pss::launch_v2_exact_draws(g, ep, h->xslot[k].p, h->xside[k]);
        if (r != hipSuccess) return r;
        return hipEventRecord(h->xev_done[k], h->xside[k]);
    };
    for (int d = 1; d <= depth && d < NX; d++) {
        bool queued = false;
        for (const auto &p : h->xpend) queued |= p.valid && p.key == key && p.epoch == e + d;
        if (queued) continue;
        int k = -1;
        for (int j = 0; j < cap_slots && k < 0; j++) if (!h->xpend[j].valid && j != use) k = j;
        if (k < 0) break;
        if (prepare_slot(k, e + d) != hipSuccess) {
            (void)hipGetLastError();
            h->xpend[k].valid = false;
            if (h->xside[k]) (void)hipStreamSynchronize(h->xside[k]);
            h->xslot[k].release();
            (void)hipGetLastError();
            h->x_failed = true;
            return PSS_OK;
        }
        h->xpend[k] = {true, key, e + d};
        h->st_x_made++;
    }
    return PSS_OK;
}

// pss_generate's device path; ma != nullptr (V2 counter order, v2_mapped_fused shapes): the
// replay writes (file, offset) into ma's arrays instead of ids into out_dev
int generate_impl(pss_sampler *h, int32_t rank_lo, int32_t rank_hi, int64_t pos_lo, int64_t count,
                  int64_t *out_dev, void *stream, const pss::MapArgs *ma);

}  // namespace

int pss_generate(pss_sampler *h, int32_t rank_lo, int32_t rank_hi, int64_t pos_lo,
                 int64_t count, int64_t *out_dev, void *stream) {
    if (!h) return fail(PSS_EINVAL, "NULL handle");
    if (rank_lo < 0 || rank_hi > h->R || rank_lo > rank_hi) return fail(PSS_EINVAL, "bad rank range");
    if (pos_lo < 0 || count < 0) return fail(PSS_EINVAL, "bad position range");
    if (count > 0 && rank_hi > rank_lo && !out_dev) return fail(PSS_EINVAL, "out_dev is NULL");
    return generate_impl(h, rank_lo, rank_hi, pos_lo, count, out_dev, stream, nullptr);
}

namespace {

int generate_impl(pss_sampler *h, int32_t rank_lo, int32_t rank_hi, int64_t pos_lo, int64_t count,
                  int64_t *out_dev, void *stream, const pss::MapArgs *ma) {
    if (h->cpu) {
        if (!h->iterated) return fail(PSS_ESTATE, "pss_init_iter must be called before generation");
        if (rank_hi == rank_lo || count == 0 || pos_lo >= h->ns) return PSS_OK;
        CpuTimer tm{h, h->version == 1 ? pss::K_V1 : pss::K_V2_EMIT};
        pss::cpu::generate(h->geometry(), h->ranks.data(), rank_lo, rank_hi - rank_lo, pos_lo, count,
                           h->epoch, h->order_mode == PSS_ORDER_EXACT, out_dev);
        return PSS_OK;
    }
    DeviceGuard dg(h->device);
    hipStream_t s = (hipStream_t)stream;
    if (!h->iterated) return fail(PSS_ESTATE, "pss_init_iter must be called before device work");
    int rc = ensure_device(h);
    if (rc) return rc;
    const int32_t nr = rank_hi - rank_lo;
    const pss::Geometry g = h->geometry();
    // the V2 exchange replay takes its ranks' descriptors as kernel arguments: no upload kernel
    // ahead of it on the epoch path (the device table is refreshed on first other use)
    // (so does V1's one-shot kernel, counter order, up to kArgRanks ranks per call)
    const bool by_value = h->order_mode == PSS_ORDER_COUNTER && nr > 0 &&
                          (h->version == 2 ? pss::v2_ranks_by_value(g, nr, h->emit_path) : nr <= pss::kArgRanks);
    // whole V2 streams, ranks by value, the lookahead ring: no shared device state (pss_sampler)
    const bool own_state = h->version == 2 && by_value && !ma && pos_lo == 0 && count >= h->ns && lookahead_on() &&
                           h->v2_depth != 0 && pss::v2_stage_split(g, nr, h->emit_path);
    std::unique_ptr<SharedUse> su;
    if (!own_state) su.reset(new SharedUse(h, s));
    pss::RankArgs ra;
    if (by_value) {
        for (int32_t i = 0; i < nr; i++) ra.r[i] = h->ranks[rank_lo + i];
    } else {
        rc = prepare(h, s);
        if (rc) return rc;
    }
    const pss::RankArgs *rap = by_value ? &ra : nullptr;
    if (nr == 0 || count == 0 || pos_lo >= h->ns) return PSS_OK;
    const pss::Marker mk = marker_of(h);
    auto words = [](size_t bytes) { return (bytes + sizeof(uint32_t) - 1) / sizeof(uint32_t); };
    if (h->version == 1 && h->order_mode == PSS_ORDER_EXACT && g.shuffle) {
        PSS_HIP(h->d_sort.ensure(words(pss::v1_exact_ws_bytes(g, nr, pos_lo, count))));
        return generate_exact(h, g, rank_lo, nr, pos_lo, count, out_dev, s, mk);
    } else if (h->version == 1) {
        const size_t sb = pss::v1_workspace_bytes(g, nr, pos_lo, count);
        if (sb) PSS_HIP(h->d_sort.ensure(words(sb)));
        PSS_HIP(pss::launch_v1(g, h->d_ranks.p, rank_lo, nr, pos_lo, count, out_dev, h->d_sort.p, s, mk,
                               nullptr, rap));
    } else if (h->order_mode == PSS_ORDER_EXACT) {
        PSS_HIP(h->d_sort.ensure(words(pss::v2_exact_ws_bytes(g, nr))));
        return generate_exact(h, g, rank_lo, nr, pos_lo, count, out_dev, s, mk);
    } else if (lookahead_on() && h->v2_depth != 0 && pss::v2_stage_split(g, nr, h->emit_path)) {
        return generate_v2_lookahead(h, g, rank_lo, nr, pos_lo, count, out_dev, s, mk, ma, rap);
    } else {
        for (auto &p : h->pend) p.valid = false;
        h->last_valid = false;
        // a lookahead pass may still write a VAL buffer, and d_val's last reader may be a replay
        // on another stream: order this launch after both on the device (no host round trip)
        if (h->side) PSS_HIP(hipStreamWaitEvent(s, h->ev_side, 0));
        if (h->ev_read[0]) PSS_HIP(hipStreamWaitEvent(s, h->ev_read[0], 0));
        PSS_HIP(h->d_val.ensure(words(pss::v2_val_bytes(g, nr))));
        const size_t bb = pss::v2_buf_bytes(g, nr), sb = pss::v2_sort_bytes(g, nr);
        if (bb) PSS_HIP(h->d_buf.ensure(words(bb)));
        if (sb) PSS_HIP(h->d_sort.ensure(words(sb)));
        PSS_HIP(pss::launch_v2(g, h->d_ranks.p, rank_lo, nr, pos_lo, count, out_dev, h->d_val.p,
                               h->d_buf.p, h->d_sort.p, h->d_err.p, s, mk, h->emit_path,
                               pss::V2_STAGE_ALL, ma, rap));
        if (h->ev_read[0]) PSS_HIP(hipEventRecord(h->ev_read[0], s));   // last user of d_val
    }
    return PSS_OK;
}

}  // namespace

int pss_set_emit_path(pss_sampler *h, int32_t path) {
    if (!h) return fail(PSS_EINVAL, "NULL handle");
    if (path < pss::EMIT_AUTO || path > pss::EMIT_PROBE) return fail(PSS_EINVAL, "bad emit path");
    if (path == pss::EMIT_XCHG && !h->cpu) {
        DeviceGuard dg(h->device);
        int rc = ensure_device(h);
        if (rc) return rc;
        if (!pss::lds_xchg_ordered())
            return fail(PSS_ENOTSUP, "device failed the LDS exchange-order check");
    }
    h->emit_path = path;
    return PSS_OK;
}

int pss_set_order_mode(pss_sampler *h, int32_t mode) {
    if (!h) return fail(PSS_EINVAL, "NULL handle");
    if (mode != PSS_ORDER_COUNTER && mode != PSS_ORDER_EXACT) return fail(PSS_EINVAL, "bad order mode");
    if (mode == PSS_ORDER_EXACT && !h->cpu) {   // the CPU mode has no LDS bounds
        if (h->version == 1 && !pss::v1_exact_supported(h->geometry()))
            return fail(PSS_ENOTSUP, "V1 exact order needs shuffle_buffer < 2^31");
        if (h->version == 2 && !pss::v2_exact_supported(h->geometry()))
            return fail(PSS_ENOTSUP, "V2 exact order needs num_samples < 2^31 and shuffle_buffer < 2^30");
    }
    if (mode != h->order_mode && mode == PSS_ORDER_COUNTER && !h->cpu && h->dev_init) {
        // leaving the exact order: the draws made ahead and their slots go
        DeviceGuard dg(h->device);
        for (int k = 0; k < pss_sampler::kXSlots; k++) {
            if (h->xside[k]) PSS_HIP(hipStreamSynchronize(h->xside[k]));
            if (h->xev_read[k]) PSS_HIP(hipEventSynchronize(h->xev_read[k]));
            h->xpend[k].valid = false;
            h->xslot[k].release();
        }
        for (auto &x : h->xhist) x.valid = false;
    }
    h->order_mode = mode;
    return PSS_OK;
}

int pss_order_mode(const pss_sampler *h, int32_t *mode) {
    if (!h || !mode) return fail(PSS_EINVAL, "NULL argument");
    *mode = h->order_mode;
    return PSS_OK;
}

int pss_emit_path(pss_sampler *h, int32_t *path) {
    if (!h || !path) return fail(PSS_EINVAL, "NULL argument");
    if (h->cpu) { *path = 0; return PSS_OK; }   // no replay kernel in CPU mode
    if (h->emit_path != pss::EMIT_AUTO) { *path = h->emit_path; return PSS_OK; }
    DeviceGuard dg(h->device);
    int rc = ensure_device(h);
    if (rc) return rc;
    *path = pss::lds_xchg_ordered() ? pss::EMIT_XCHG : pss::EMIT_PROBE;
    return PSS_OK;
}

int pss_profile(pss_sampler *h, int32_t enable) {
    if (!h) return fail(PSS_EINVAL, "NULL handle");
    if (enable < 0) return fail(PSS_EINVAL, "profile mode must be >= 0");
    h->profiling = enable != 0;
    h->profile_mode = enable;
    h->prof_seen = 0;
    h->spans.clear();
    h->ev_used = 0;
    h->open_kind = -1;
    return PSS_OK;
}

int pss_profile_read(pss_sampler *h, double *total_ms, int64_t *launches, int32_t nkinds) {
    if (!h || !total_ms || !launches) return fail(PSS_EINVAL, "NULL argument");
    for (int32_t k = 0; k < nkinds; k++) { total_ms[k] = 0; launches[k] = 0; }
    if (h->cpu) {
        for (int32_t k = 0; k < nkinds && k < pss::K_NUM_KINDS; k++) {
            total_ms[k] = h->cpu_ms[k];
            launches[k] = h->cpu_calls[k];
            h->cpu_ms[k] = 0;
            h->cpu_calls[k] = 0;
        }
        return PSS_OK;
    }
    DeviceGuard dg(h->device);
    for (const auto &sp : h->spans) {
        PSS_HIP(hipEventSynchronize(h->ev_pool[sp.b]));
        float ms = 0.f;
        PSS_HIP(hipEventElapsedTime(&ms, h->ev_pool[sp.a], h->ev_pool[sp.b]));
        if (sp.kind >= 0 && sp.kind < nkinds) { total_ms[sp.kind] += ms; launches[sp.kind] += 1; }
    }
    h->spans.clear();
    h->ev_used = 0;
    h->open_kind = -1;
    return PSS_OK;
}

int pss_map(pss_sampler *h, const int64_t *ids_dev, int64_t n, int32_t *file_pos_dev,
            int64_t *offset_dev, void *stream) {
    if (!h) return fail(PSS_EINVAL, "NULL handle");
    if (n < 0 || (n > 0 && (!ids_dev || !file_pos_dev || !offset_dev))) return fail(PSS_EINVAL, "bad arguments");
    if (h->F == 0) return fail(PSS_ESTATE, "no files to map into");
    if (h->cpu) {
        const int rc = cpu_prefix(h);
        if (rc) return rc;
        CpuTimer tm{h, pss::K_MAP};
        pss::cpu::map(h->h_prefix.data(), h->F, ids_dev, n, file_pos_dev, offset_dev);
        return PSS_OK;
    }
    DeviceGuard dg(h->device);
    hipStream_t s = (hipStream_t)stream;
    SharedUse su(h, s);
    int rc = prepare_tables(h, s);
    if (rc) return rc;
    const pss_sampler::TabSet &t = h->tab[h->tab_cur];
    PSS_HIP(pss::launch_map(t.prefix, h->F, t.bucket, h->kb, h->nb, ids_dev, n, file_pos_dev,
                            offset_dev, nullptr, s));
    return tables_read(h, s);
}

// pss_generate_mapped's device work after the epoch's tables are ready on s
static int generate_mapped_dev(pss_sampler *h, int32_t rank_lo, int32_t rank_hi, int64_t pos_lo,
                               int64_t count, int32_t *file_pos_dev, int32_t *offset_dev, hipStream_t s);

int pss_generate_mapped(pss_sampler *h, int32_t rank_lo, int32_t rank_hi, int64_t pos_lo,
                        int64_t count, int32_t *file_pos_dev, int32_t *offset_dev, void *stream) {
    if (!h) return fail(PSS_EINVAL, "NULL handle");
    if (rank_lo < 0 || rank_hi > h->R || rank_lo > rank_hi) return fail(PSS_EINVAL, "bad rank range");
    if (pos_lo < 0 || count < 0) return fail(PSS_EINVAL, "bad position range");
    if (count > 0 && rank_hi > rank_lo && (!file_pos_dev || !offset_dev)) return fail(PSS_EINVAL, "NULL output");
    if (h->F == 0) return fail(PSS_ESTATE, "no files to map into");
    if (h->max_len > (int64_t)INT32_MAX) return fail(PSS_ENOTSUP, "a file longer than 2^31-1 samples (int32 offsets)");
    const int32_t nr = rank_hi - rank_lo;
    if (nr == 0 || count == 0 || pos_lo >= h->ns) return PSS_OK;
    const size_t n = (size_t)nr * (size_t)count;
    if (h->cpu) {
        const int rc = cpu_prefix(h);
        if (rc) return rc;
        std::vector<int64_t> ids(n, 0), off(n);
        int rc2 = pss_generate(h, rank_lo, rank_hi, pos_lo, count, ids.data(), nullptr);
        if (rc2) return rc2;
        const int64_t valid = std::min(count, h->ns - pos_lo);
        CpuTimer tm{h, pss::K_MAP};
        for (int32_t r = 0; r < nr; r++) {
            const size_t o = (size_t)r * count;
            pss::cpu::map(h->h_prefix.data(), h->F, ids.data() + o, valid, file_pos_dev + o, off.data() + o);
            for (int64_t i = 0; i < valid; i++) offset_dev[o + i] = (int32_t)off[o + i];
        }
        return PSS_OK;
    }
    DeviceGuard dg(h->device);
    hipStream_t s = (hipStream_t)stream;
    SharedUse su(h, s);
    int rc = prepare_tables(h, s);
    if (rc) return rc;
    rc = generate_mapped_dev(h, rank_lo, rank_hi, pos_lo, count, file_pos_dev, offset_dev, s);
    return rc ? rc : tables_read(h, s);
}

static int generate_mapped_dev(pss_sampler *h, int32_t rank_lo, int32_t rank_hi, int64_t pos_lo,
                               int64_t count, int32_t *file_pos_dev, int32_t *offset_dev, hipStream_t s) {
    const int32_t nr = rank_hi - rank_lo;
    const size_t n = (size_t)nr * (size_t)count;
    void *stream = (void *)s;
    int rc = PSS_OK;
    const pss::Geometry g = h->geometry();
    const pss::Marker mk = marker_of(h);
    auto words = [](size_t bytes) { return (bytes + sizeof(uint32_t) - 1) / sizeof(uint32_t); };
    const bool exact = h->order_mode == PSS_ORDER_EXACT && (h->version == 2 || g.shuffle);
    if (h->version == 1 && !exact) {
        // fused: the V1 kernel maps each id as it computes it (shuffle = false is the identity
        // order of both modes); up to kArgRanks ranks' descriptors by value (no upload kernel)
        const size_t sb = pss::v1_workspace_bytes(g, nr, pos_lo, count);
        if (sb) PSS_HIP(h->d_sort.ensure(words(sb)));
        const pss::MapArgs ma = map_args(h, file_pos_dev, offset_dev);
        pss::RankArgs ra;
        const bool by_value = nr <= pss::kArgRanks;
        if (by_value) {
            for (int32_t i = 0; i < nr; i++) ra.r[i] = h->ranks[rank_lo + i];
        } else if ((rc = prepare(h, s)) != PSS_OK) {
            return rc;
        }
        PSS_HIP(pss::launch_v1(g, h->d_ranks.p, rank_lo, nr, pos_lo, count, nullptr, h->d_sort.p, s, mk, &ma,
                               by_value ? &ra : nullptr));
        return PSS_OK;
    }
    if (exact) {
        // fused: the exact pipelines' output kernels map each id where they would write it
        if ((rc = prepare(h, s)) != PSS_OK) return rc;
        const pss::MapArgs ma = map_args(h, file_pos_dev, offset_dev);
        if (h->version == 1) {
            PSS_HIP(h->d_sort.ensure(words(pss::v1_exact_ws_bytes(g, nr, pos_lo, count))));
            mk(pss::K_V1, s);
            PSS_HIP(pss::launch_v1_exact(g, h->d_ranks.p, rank_lo, nr, pos_lo, count, h->epoch, nullptr,
                                         h->d_sort.p, s, &ma));
        } else {
            PSS_HIP(h->d_sort.ensure(words(pss::v2_exact_ws_bytes(g, nr))));
            mk(pss::K_V2_EMIT, s);
            PSS_HIP(pss::launch_v2_exact(g, h->d_ranks.p, rank_lo, nr, pos_lo, count, h->epoch, nullptr,
                                         h->d_sort.p, s, &ma));
        }
        mk(-1, s);
        return PSS_OK;
    }
    if (h->version == 2 && h->order_mode == PSS_ORDER_COUNTER && pss::v2_mapped_fused(g, h->emit_path)) {
        // fused: the replay maps each id as it emits it (LDS segment map per tile)
        const pss::MapArgs ma = map_args(h, file_pos_dev, offset_dev);
        return generate_impl(h, rank_lo, rank_hi, pos_lo, count, nullptr, stream, &ma);
    }
    // the V2 collision-probe path: ids into the handle's scratch, then the bucket map
    if (!h->ids_free) PSS_HIP(hipEventCreateWithFlags(&h->ids_free, hipEventDisableTiming));
    if (h->d_ids.n < n) {
        PSS_HIP(hipEventSynchronize(h->ids_free));
        PSS_HIP(h->d_ids.ensure(n));
    }
    PSS_HIP(hipStreamWaitEvent(s, h->ids_free, 0));
    rc = pss_generate(h, rank_lo, rank_hi, pos_lo, count, h->d_ids.p, stream);
    if (rc) return rc;
    const int64_t valid = std::min(count, h->ns - pos_lo);
    mk(pss::K_MAP, s);
    const pss_sampler::TabSet &t = h->tab[h->tab_cur];
    for (int32_t r = 0; r < nr; r++) {
        const size_t o = (size_t)r * count;
        PSS_HIP(pss::launch_map(t.prefix, h->F, t.bucket, h->kb, h->nb, h->d_ids.p + o, valid,
                                file_pos_dev + o, nullptr, offset_dev + o, s));
    }
    mk(-1, s);
    PSS_HIP(hipEventRecord(h->ids_free, s));
    return PSS_OK;
}

int pss_gather(pss_sampler *h, const void *data_dev, int64_t row_bytes, const int64_t *base_rows_dev,
               const int32_t *file_pos_dev, const int32_t *offset_dev, int64_t n, void *out_dev,
               void *stream) {
    if (!h) return fail(PSS_EINVAL, "NULL handle");
    if (n < 0 || row_bytes < 0 || (n > 0 && (!data_dev || !base_rows_dev || !file_pos_dev || !offset_dev || !out_dev)))
        return fail(PSS_EINVAL, "bad arguments");
    if (n == 0 || row_bytes == 0) return PSS_OK;
    if (h->cpu) {
        const char *d = (const char *)data_dev;
        char *o = (char *)out_dev;
        for (int64_t i = 0; i < n; i++) {
            const int32_t f = file_pos_dev[i] < 0 ? -1 - file_pos_dev[i] : file_pos_dev[i];
            const int64_t row = base_rows_dev[h->order[f]] + offset_dev[i];
            std::memcpy(o + i * row_bytes, d + row * row_bytes, (size_t)row_bytes);
        }
        return PSS_OK;
    }
    DeviceGuard dg(h->device);
    hipStream_t s = (hipStream_t)stream;
    SharedUse su(h, s);
    const int rc = prepare_tables(h, s);
    if (rc) return rc;
    PSS_HIP(pss::launch_gather(data_dev, row_bytes, base_rows_dev, h->tab[h->tab_cur].order, file_pos_dev,
                               offset_dev, n, out_dev, s));
    return tables_read(h, s);
}

int pss_partition(pss_sampler *h, int32_t rank_lo, int32_t rank_hi, int64_t *seg_off_dev,
                  int32_t *seg_file_dev, int64_t *seg_lo_dev, int64_t *seg_hi_dev,
                  int64_t seg_cap, void *stream) {
    if (!h) return fail(PSS_EINVAL, "NULL handle");
    if (rank_lo < 0 || rank_hi > h->R || rank_lo > rank_hi) return fail(PSS_EINVAL, "bad rank range");
    if (!seg_off_dev) return fail(PSS_EINVAL, "seg_off_dev is NULL");
    if (seg_cap > 0 && (!seg_file_dev || !seg_lo_dev || !seg_hi_dev)) return fail(PSS_EINVAL, "NULL segment arrays");
    if (h->F == 0) return fail(PSS_ESTATE, "no files to partition");
    if (h->cpu) {
        const int rc = cpu_prefix(h);
        if (rc) return rc;
        if (!pss::cpu::partition(h->geometry(), h->ranks.data(), rank_lo, rank_hi - rank_lo, h->h_prefix.data(),
                                 h->F, seg_off_dev, seg_file_dev, seg_lo_dev, seg_hi_dev, seg_cap))
            return fail(PSS_EDEVICE, "partition capacity exceeded");
        return PSS_OK;
    }
    DeviceGuard dg(h->device);
    hipStream_t s = (hipStream_t)stream;
    SharedUse su(h, s);
    int rc = prepare(h, s);
    if (rc == PSS_OK) rc = prepare_tables(h, s);
    if (rc) return rc;
    PSS_HIP(pss::launch_partition(h->geometry(), h->d_ranks.p, rank_lo, rank_hi - rank_lo,
                                  h->tab[h->tab_cur].prefix, h->F, seg_off_dev, seg_file_dev, seg_lo_dev,
                                  seg_hi_dev, seg_cap, h->d_err.p, s));
    return tables_read(h, s);
}

int pss_digest(const int64_t *ids_dev, int64_t n, uint64_t *acc_dev, void *stream) {
    if (n < 0 || (n > 0 && (!ids_dev || !acc_dev))) return fail(PSS_EINVAL, "bad arguments");
    PSS_HIP(pss::launch_digest(ids_dev, n, acc_dev, (hipStream_t)stream));
    return PSS_OK;
}

int pss_digest_range(int64_t lo, int64_t hi, uint64_t *acc_dev, void *stream) {
    if (!acc_dev) return fail(PSS_EINVAL, "acc_dev is NULL");
    PSS_HIP(pss::launch_digest_range(lo, hi, acc_dev, (hipStream_t)stream));
    return PSS_OK;
}

int pss_set_lookahead(pss_sampler *h, int32_t exact_depth, int64_t exact_max_bytes, int32_t v2_depth) {
    if (!h) return fail(PSS_EINVAL, "NULL handle");
    if (exact_depth < -1 || exact_depth > pss_sampler::kXSlots - 1) return fail(PSS_EINVAL, "exact_depth must be -1 .. 8");
    if (exact_max_bytes < 0) return fail(PSS_EINVAL, "exact_max_bytes must be >= 0");
    if (v2_depth < -1 || v2_depth > 2) return fail(PSS_EINVAL, "v2_depth must be -1 .. 2");
    if (v2_depth != h->v2_depth) {
        // queued passes were sized and keyed for the previous depth: drop them (their buffers
        // stay, ordered by their events)
        for (auto &p : h->pend) p.valid = false;
        h->last_valid = false;
    }
    h->x_depth = exact_depth;
    h->x_cap = exact_max_bytes;
    h->v2_depth = v2_depth;
    h->x_failed = false;
    return PSS_OK;
}

int pss_lookahead_stats(const pss_sampler *h, int64_t *stats) {
    if (!h || !stats) return fail(PSS_EINVAL, "NULL argument");
    stats[0] = h->st_x_made;
    stats[1] = h->st_x_used;
    stats[2] = h->st_v2_queued;
    stats[3] = h->st_v2_used;
    return PSS_OK;
}

int pss_workspace_bytes(const pss_sampler *h, int64_t *bytes) {
    if (!h || !bytes) return fail(PSS_EINVAL, "NULL argument");
    int64_t b = 0;
    auto add = [&](const auto &d) { b += (int64_t)(d.n * sizeof(*d.p)); };
    add(h->d_lens); add(h->d_ids); add(h->d_ranks); add(h->d_err);
    add(h->d_val); add(h->d_buf); add(h->d_sort);
    add(h->d_val2); add(h->d_buf2); add(h->d_val3); add(h->d_buf3);
    for (const auto &t : h->tab) add(t.blob);
    for (const auto &x : h->xslot) add(x);
    *bytes = b;
    return PSS_OK;
}

int pss_check(pss_sampler *h, void *stream) {
    if (!h) return fail(PSS_EINVAL, "NULL handle");
    if (h->cpu) return PSS_OK;   // CPU mode reports errors by return code
    DeviceGuard dg(h->device);
    PSS_HIP(hipStreamSynchronize((hipStream_t)stream));
    // lookahead passes on the side stream share the error word: let them land first
    if (h->side) PSS_HIP(hipStreamSynchronize(h->side));
    PSS_HIP(hipGetLastError());
    if (!h->dev_init) return PSS_OK;
    int32_t err = 0;
    PSS_HIP(hipMemcpy(&err, h->d_err.p, sizeof(int32_t), hipMemcpyDeviceToHost));
    if (err) {
        PSS_HIP(hipMemset(h->d_err.p, 0, sizeof(int32_t)));
        return fail(PSS_EDEVICE, "device error flag " + std::to_string(err) +
                                     " (1: partition capacity exceeded, 2: sort bucket overflow)");
    }
    return PSS_OK;
}

int pss_error_snapshot(pss_sampler *h, int32_t *dst, void *stream) {
    if (!h || !dst) return fail(PSS_EINVAL, "NULL argument");
    if (h->cpu || !h->dev_init) { *dst = 0; return PSS_OK; }
    DeviceGuard dg(h->device);
    // not ordered after queued lookahead passes (that would hold the caller's stream behind
    // the next epochs' work): a flag they raise shows in a later snapshot or in pss_check
    PSS_HIP(hipMemcpyAsync(dst, h->d_err.p, sizeof(int32_t), hipMemcpyDeviceToHost, (hipStream_t)stream));
    return PSS_OK;
}

int pss_map_prefix_host(const int64_t *prefix, int64_t nfiles, const int64_t *ids, int64_t n,
                        int32_t *file_pos, int64_t *offset) {
    if (nfiles < 0 || n < 0 || !prefix || (n > 0 && (!ids || !file_pos || !offset)))
        return fail(PSS_EINVAL, "bad arguments");
    if (nfiles == 0) return fail(PSS_ESTATE, "no files to map into");
    pss::cpu::map(prefix, nfiles, ids, n, file_pos, offset);
    return PSS_OK;
}

int pss_digest_host(const int64_t *ids, int64_t n, uint64_t *acc) {
    if (n < 0 || !acc || (n > 0 && !ids)) return fail(PSS_EINVAL, "bad arguments");
    *acc += pss::cpu::digest(ids, n);
    return PSS_OK;
}

int pss_digest_range_host(int64_t lo, int64_t hi, uint64_t *acc) {
    if (!acc) return fail(PSS_EINVAL, "acc is NULL");
    *acc += pss::cpu::digest_range(lo, hi);
    return PSS_OK;
}

int pss_device(const pss_sampler *h, int32_t *device) {
    if (!h || !device) return fail(PSS_EINVAL, "NULL argument");
    *device = h->cpu ? PSS_DEVICE_CPU : h->device;
    return PSS_OK;
}

int pss_debug_wave_scan(const uint64_t *in_dev, uint64_t *out_dev, int64_t n, void *stream) {
    if (n <= 0 || !in_dev || !out_dev) return fail(PSS_EINVAL, "bad arguments");
    PSS_HIP(pss::launch_debug_wave_scan(in_dev, out_dev, n, (hipStream_t)stream));
    return PSS_OK;
}

}  // extern "C"
