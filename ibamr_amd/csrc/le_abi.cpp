// le_abi.cpp -- the C-ABI of include/ibtk_le.h: contexts, marker binning and
// the interp/spread entry points over device-resident data.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdlib>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/ibtk_le.h"
#include "le_internal.h"

using namespace ibtk_le;

// ---------------------------------------------------------------------------
// errors
// ---------------------------------------------------------------------------
static thread_local std::string g_last_error;

static int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_last_error = buf;
    return code;
}

#define HIP_TRY(expr)                                                                                     \
    do {                                                                                                  \
        hipError_t _e = (expr);                                                                           \
        if (_e != hipSuccess) return fail(IBTK_LE_ERR_DEVICE, "%s: %s", #expr, hipGetErrorString(_e));    \
    } while (0)

extern "C" const char* ibtk_le_last_error(void) { return g_last_error.c_str(); }
extern "C" const char* ibtk_le_version(void) { return "ibtk_le 0.1 (gfx950)"; }

// ---------------------------------------------------------------------------
// kernel names (LEInteractor::getStencilSize, LEInteractor.cpp:668-682)
// ---------------------------------------------------------------------------
static const char* const kNames[K_COUNT] = {"PIECEWISE_CONSTANT", "DISCONTINUOUS_LINEAR", "PIECEWISE_LINEAR",
                                            "PIECEWISE_CUBIC",    "IB_3",                 "IB_4",
                                            "IB_4_W8",            "IB_6",                 "BSPLINE_4"};
static const int kStencil[K_COUNT] = {1, 2, 2, 4, 4, 4, 8, 6, 4};

// USER_DEFINED (LEInteractor.cpp:651-652): the user's kernel function and its
// stencil size, IB_4's by default (ib4_kernel_fcn, LEInteractor.cpp:629-648)
extern "C" double ibtk_le_ib4_kernel_fcn(double r) {
    r = std::abs(r);
    if (r < 1.0) {
        const double t2 = r * r;
        const double t6 = std::sqrt(-0.4e1 * t2 + 0.4e1 * r + 0.1e1);
        return -r / 0.4e1 + 0.3e1 / 0.8e1 + t6 / 0.8e1;
    } else if (r < 2.0) {
        const double t2 = r * r;
        const double t6 = std::sqrt(0.12e2 * r - 0.7e1 - 0.4e1 * t2);
        return -r / 0.4e1 + 0.5e1 / 0.8e1 - t6 / 0.8e1;
    }
    return 0.0;
}
static ibtk_le_user_kernel_fn g_user_fcn = &ibtk_le_ib4_kernel_fcn;
static int g_user_size = 4;
// Any stencil size (LEInteractor.cpp:652, 678): the per-entry weight tables are sized
// from it at the call; only the spread's 32-bit contribution count limits n S^NDIM
// (checked there).  This bound keeps S^3 itself inside an int.
constexpr int USER_MAX_STENCIL = 1024;

extern "C" int ibtk_le_set_user_kernel(ibtk_le_user_kernel_fn fcn, int stencil_size) {
    if (stencil_size < 1 || stencil_size > USER_MAX_STENCIL)
        return fail(IBTK_LE_ERR_ARG, "user kernel stencil size %d outside [1, %d]", stencil_size, USER_MAX_STENCIL);
    g_user_fcn = fcn ? fcn : &ibtk_le_ib4_kernel_fcn;
    g_user_size = stencil_size;
    return IBTK_LE_OK;
}
extern "C" int ibtk_le_user_kernel(ibtk_le_user_kernel_fn* fcn, int* stencil_size) {
    if (fcn) *fcn = g_user_fcn;
    if (stencil_size) *stencil_size = g_user_size;
    return IBTK_LE_OK;
}

extern "C" int ibtk_le_kernel_from_name(const char* name) {
    if (!name) return -1;
    for (int k = 0; k < K_COUNT; ++k)
        if (std::strcmp(name, kNames[k]) == 0) return k;
    if (std::strcmp(name, "USER_DEFINED") == 0) return IBTK_LE_KERNEL_USER_DEFINED;
    return -1;
}
extern "C" const char* ibtk_le_kernel_name(int kernel) {
    if (kernel == IBTK_LE_KERNEL_USER_DEFINED) return "USER_DEFINED";
    return (kernel >= 0 && kernel < K_COUNT) ? kNames[kernel] : nullptr;
}
extern "C" int ibtk_le_stencil_size(int kernel) {
    if (kernel == IBTK_LE_KERNEL_USER_DEFINED) return g_user_size;
    return (kernel >= 0 && kernel < K_COUNT) ? kStencil[kernel] : -1;
}
extern "C" int ibtk_le_min_ghost_width(int kernel) {
    // LEInteractor.cpp:684-687: floor(0.5*stencil) + 1
    const int s = ibtk_le_stencil_size(kernel);
    return s < 0 ? -1 : s / 2 + 1;
}

// ---------------------------------------------------------------------------
// device buffers
// ---------------------------------------------------------------------------
struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    int ensure(size_t bytes) {
        if (bytes <= cap) return IBTK_LE_OK;
        if (p) hipFree(p);
        p = nullptr;
        cap = 0;
        size_t want = bytes + bytes / 8 + 256;
        if (hipMalloc(&p, want) != hipSuccess) {
            p = nullptr;
            return fail(IBTK_LE_ERR_NOMEM, "hipMalloc(%zu) failed", want);
        }
        cap = want;
        return IBTK_LE_OK;
    }
    void release() {
        if (p) hipFree(p);
        p = nullptr;
        cap = 0;
    }
    template <class T> T* as() const { return static_cast<T*>(p); }
};

struct ibtk_le_ctx_s {
    int device = 0;
    hipStream_t stream = nullptr;
    DevBuf keys_in, vals_in, temp, counts, offsets, fbuf;
    DevBuf bfirst;  // first entry of every bucket (k_gather_col), before the suffix-min scan
    DevBuf usr_lo, usr_cnt, usr_w, usr_s, usr_last, usr_x0, usr_x1;  // USER_DEFINED tables
    DevBuf lst_idx, lst_xs, lst_key, lst_perm;  // index-list / node-distribution scratch
    DevBuf lst_cell, lst2_idx, lst2_xs, lst2_cell, lst_flag;  // index lists: cells, the sorted list, unique flags
    DevBuf num_tab, num_lkey, num_ckey;                        // level numbering: tile table, keys
    DevBuf ll_cnt, ll_key, ll_key2, ll_id, ll_id2, ll_src, ll_img, ll_off;  // level index lists
    DevBuf lvl_tab;                             // level ghost fill tables
    std::vector<char> lvl_host;                 // what lvl_tab holds
    DevBuf zero_tab;                            // level zero tables
    std::vector<char> zero_host;                // what zero_tab holds
    DevBuf err;   // one int
    DevBuf sink;  // 64 doubles (Params::sink)
    DevBuf stamps;  // diagnostic phase clocks (IBTK_LE_STAMPS=1)
    DevBuf mig_cls, mig_cnt;  // ibtk_le_slab_update_partition scratch
    bool stamps_on = false;  // IBTK_LE_STAMPS=1, read once at ctx_create
    bool count_adds = false; // ibtk_le_ctx_count_adds: the spread sweeps count their ds_add_f64
    DevBuf adds;             // the device counters
    unsigned long long last_adds[2] = {0, 0};
    SweepTune tune;          // ibtk_le_ctx_tune (diagnostics)
    int zmode = 0, zlo = 0, zhi = -1;  // ibtk_le_ctx_set_plane_window
    bool timing = false;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    bool ev_valid = false;
    // the 3-D spread's F gather runs on a side stream, concurrent with the candidate-stream
    // rebuild on `stream` (gather_fork / gather_join), created on first use
    hipStream_t side = nullptr;
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    // pinned host staging of small read-backs (d2h_sync): a copy into pageable memory is a
    // staged, blocking copy of its own
    void* hstage = nullptr;
    size_t hstage_cap = 0;
};

struct ibtk_le_markers_s {
    ibtk_le_ctx ctx = nullptr;
    int n = 0;
    int kernel = -1;
    int ndim = 0;
    BinGeom bg{};
    ColGeom cg{};        // 3-D: column binning (le_sweep.hip)
    int S = 0, nseg = 0;  // 3-D: sweep segments
    ibtk_le_patch_geom geom{};
    DevBuf sorted_key, sorted_l, sorted_s, sorted_X, sorted_a, plane_start, indices, xshift;
    // 3-D: the sorted positions are sorted_X or sorted_X2, the one the device cell xcur
    // names (ibtk_le_markers_rebin swaps them on the device); xcur_set once it is written
    DevBuf sorted_X2, xcur;
    bool xcur_set = false;
    DevBuf lvl_nbr;                     // ibtk_le_level_fill_interp's neighbour table ...
    std::vector<int2> lvl_nbr_host;     // ... and what it holds
    DevBuf cand_cnt, cand_off, cand_idx;  // spread candidate lists, built on first use after a bin
    DevBuf last, qdst;                    // interp with duplicate list entries (Params::qdst)
    DevBuf items, nsub, isub, nitems;     // 3-D sweep item table
    // the 3-D spread's candidate stream (launch_cand_stream), built on the first spread after
    // a binning: 0 stale, 1 built, 2 stale unless the last re-binning moved nothing (the
    // build then skips on the device, cs_skip = that re-binning's mover count)
    DevBuf cs_cnt, cs_off, cs_pos;
    int cs_state = 0;
    const int* cs_skip = nullptr;
    // closed-form kernels: the stream split by the shifted-z anchor and its boundaries in
    // that frame (cs_off_z, nclz = Σ ncol (nz + 1) + 1 entries) -- built with the stream
    // when a spread's components need them (cs_split)
    DevBuf cs_off_z;
    bool cs_split = false;
    long long nclz = 0;
    // the re-binning's shifted-z anchor parities and their state (RebinBufs::zbits, zst)
    DevBuf zbits, zst;
    int rb_epoch = 0;  // re-binnings so far (RebinBufs::epoch)
    int item_bound = 0;
    // a level of patches (ibtk_le_level_bin): 0 = one patch (the fields above)
    int npatch = 0;
    std::vector<ibtk_le_patch_geom> geoms;
    std::vector<PatchDesc> pdh;           // host copy of the patch table (comps filled per call)
    std::vector<PatchDesc> pdh_dev;       // what the device table holds (uploads skipped when unchanged)
    std::vector<int> off_dev;             // what entry_off holds
    DevBuf pd, entry_off;
    int nbuckets_total = 0, njobs = 0;
    bool has_indices = false, has_xshift = false;
    bool cand_valid = false;
    bool dedup_done = false, has_dups = false;
    DevBuf qin, owner, int_off;           // ibtk_le_level_select_interior: per sorted entry, its Q target or -1
    bool qin_valid = false;               // cleared by every bin
    // the selection's cache: a re-binning in which nothing moved keeps the order, and then
    // the selection of the same interior lists stands (the lists are the binned lists' own,
    // fixed between binnings as ibtk_le_markers_rebin takes them to be).  sel_gs = {order
    // generation (bumped by k_rebin_commit when something moved), the selection's}; a full
    // binning clears sel_cached
    DevBuf sel_gs;
    bool sel_cached = false;
    std::vector<int> sel_off;
    const int* sel_idx = nullptr;
    int sel_nm = -1;
    // ibtk_le_markers_rebin: the last binning's list (n_dev of a fixed-capacity one) and its scratch
    const int* n_dev = nullptr;
    bool binned3 = false;                 // a 3-D column binning (ibtk_le_markers_bin(_count) / level_bin) holds
    DevBuf rb_cin, rb_cout, rb_d, rb_dpre, rb_mstart, rb_ps2, rb_mbits, rb_wcnt, rb_wpre, rb_mlist, rb_scr, rb_big,
        rb_nbig;
    int rb_zeroed_nb = -1;                // rb_cin / rb_cout are zero for this many buckets
    int items_sig[12] = {-1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};  // what the item table was built with (cuts, strip, target, heavy)
};

static int set_device(ibtk_le_ctx ctx) {
    HIP_TRY(hipSetDevice(ctx->device));
    return IBTK_LE_OK;
}

extern "C" int ibtk_le_ctx_create(int device, void* stream, ibtk_le_ctx* out) {
    if (!out) return fail(IBTK_LE_ERR_ARG, "ctx_create: null out");
    int ndev = 0;
    HIP_TRY(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return fail(IBTK_LE_ERR_ARG, "ctx_create: device %d of %d", device, ndev);
    auto* c = new ibtk_le_ctx_s();
    c->device = device;
    c->stream = static_cast<hipStream_t>(stream);
    if (const char* e = getenv("IBTK_LE_STAMPS")) c->stamps_on = e[0] == '1';
    HIP_TRY(hipSetDevice(device));
    int rc = c->err.ensure(sizeof(int));
    if (!rc) rc = c->sink.ensure(64 * sizeof(double));
    if (rc) {
        delete c;
        return rc;
    }
    HIP_TRY(hipMemsetAsync(c->err.p, 0, sizeof(int), c->stream));
    HIP_TRY(hipEventCreate(&c->ev0));
    HIP_TRY(hipEventCreate(&c->ev1));
    *out = c;
    return IBTK_LE_OK;
}

extern "C" int ibtk_le_ctx_destroy(ibtk_le_ctx ctx) {
    if (!ctx) return IBTK_LE_OK;
    hipSetDevice(ctx->device);
    hipStreamSynchronize(ctx->stream);
    for (DevBuf* b : {&ctx->keys_in, &ctx->vals_in, &ctx->bfirst, &ctx->usr_lo, &ctx->usr_cnt, &ctx->usr_w, &ctx->usr_s,
                      &ctx->usr_last, &ctx->usr_x0, &ctx->usr_x1, &ctx->temp, &ctx->counts, &ctx->offsets, &ctx->fbuf, &ctx->err, &ctx->sink,
                       &ctx->stamps, &ctx->lst_idx, &ctx->lst_xs, &ctx->lst_key, &ctx->lst_perm, &ctx->lst_cell,
                       &ctx->lst2_idx, &ctx->lst2_xs, &ctx->lst2_cell, &ctx->lst_flag, &ctx->num_tab, &ctx->num_lkey,
                       &ctx->num_ckey, &ctx->ll_cnt, &ctx->ll_key, &ctx->ll_key2, &ctx->ll_id, &ctx->ll_id2,
                       &ctx->ll_src, &ctx->ll_img, &ctx->ll_off,
                       &ctx->lvl_tab, &ctx->zero_tab, &ctx->mig_cls, &ctx->mig_cnt, &ctx->adds})
        b->release();
    if (ctx->ev0) hipEventDestroy(ctx->ev0);
    if (ctx->ev1) hipEventDestroy(ctx->ev1);
    if (ctx->side) {
        hipStreamSynchronize(ctx->side);
        hipStreamDestroy(ctx->side);
    }
    if (ctx->ev_fork) hipEventDestroy(ctx->ev_fork);
    if (ctx->ev_join) hipEventDestroy(ctx->ev_join);
    if (ctx->hstage) hipHostFree(ctx->hstage);
    delete ctx;
    return IBTK_LE_OK;
}

extern "C" int ibtk_le_ctx_set_stream(ibtk_le_ctx ctx, void* stream) {
    if (!ctx) return fail(IBTK_LE_ERR_ARG, "null ctx");
    ctx->stream = static_cast<hipStream_t>(stream);
    return IBTK_LE_OK;
}

extern "C" int ibtk_le_ctx_synchronize(ibtk_le_ctx ctx) {
    if (!ctx) return fail(IBTK_LE_ERR_ARG, "null ctx");
    if (set_device(ctx)) return IBTK_LE_ERR_DEVICE;
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    int flag = 0;
    HIP_TRY(hipMemcpy(&flag, ctx->err.p, sizeof(int), hipMemcpyDeviceToHost));
    if (flag) {
        HIP_TRY(hipMemset(ctx->err.p, 0, sizeof(int)));
        return fail(IBTK_LE_ERR_INVARIANT,
                    "device invariant failed (flag %d): a stencil left its staged region (1) or its bin bounds (2), "
                    "an interior list entry is not in the level's binned lists (4), a fixed-capacity "
                    "migration overflowed (8), or the spread's candidate stream reached 2^31 entries (16)",
                    flag);
    }
    return IBTK_LE_OK;
}

extern "C" int ibtk_le_ctx_set_plane_window(ibtk_le_ctx ctx, int mode, int zlo, int zhi) {
    if (!ctx) return fail(IBTK_LE_ERR_ARG, "null ctx");
    if (mode < 0 || mode > 2) return fail(IBTK_LE_ERR_ARG, "plane window mode: 0 all, 1 inside, 2 outside");
    ctx->zmode = mode;
    ctx->zlo = zlo;
    ctx->zhi = zhi;
    return IBTK_LE_OK;
}

extern "C" int ibtk_le_ctx_tune(ibtk_le_ctx ctx, const char* key, int value) {
    if (!ctx || !key) return fail(IBTK_LE_ERR_ARG, "null argument");
    SweepTune& t = ctx->tune;
    const std::string k = key;
    if (k == "seg_items") t.seg_items = value;
    else if (k == "split_target") t.split_target = value;
    else if (k == "heavy") t.heavy = value;
    else if (k == "min_piece") t.min_piece = value;
    else if (k == "heavy_target") t.heavy_target = value;
    else if (k == "heavy_min_piece") t.heavy_min_piece = value;
    else if (k == "heavy_first") t.heavy_first = value;
    else if (k == "strip") t.strip = value;
    else if (k == "xcd_block") t.xcd_block = value;
    else if (k == "interp3") t.interp3 = value;
    else if (k == "side_gather") t.side_gather = value;
    else return fail(IBTK_LE_ERR_ARG, "unknown tuning key %s", key);
    return IBTK_LE_OK;
}

extern "C" int ibtk_le_ctx_enable_timing(ibtk_le_ctx ctx, int enable) {
    if (!ctx) return fail(IBTK_LE_ERR_ARG, "null ctx");
    ctx->timing = enable != 0;
    return IBTK_LE_OK;
}

extern "C" double ibtk_le_ctx_last_kernel_ms(ibtk_le_ctx ctx) {
    if (!ctx || !ctx->ev_valid) return -1.0;
    hipEventSynchronize(ctx->ev1);
    float ms = -1.f;
    if (hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1) != hipSuccess) return -1.0;
    return ms;
}

// ---------------------------------------------------------------------------
// geometry helpers
// ---------------------------------------------------------------------------
static int check_geom(const ibtk_le_patch_geom* g) {
    if (!g) return fail(IBTK_LE_ERR_ARG, "null geometry");
    if (g->ndim != 2 && g->ndim != 3) return fail(IBTK_LE_ERR_ARG, "ndim must be 2 or 3 (got %d)", g->ndim);
    for (int d = 0; d < g->ndim; ++d) {
        if (g->iupper[d] < g->ilower[d]) return fail(IBTK_LE_ERR_ARG, "empty patch box in dim %d", d);
        if (g->gcw[d] < 0) return fail(IBTK_LE_ERR_ARG, "negative ghost width");
        if (!(g->dx[d] > 0.0)) return fail(IBTK_LE_ERR_ARG, "dx[%d] must be positive", d);
    }
    if (g->pitch[0] || g->pitch[1]) {
        if (g->ndim != 3) return fail(IBTK_LE_ERR_ARG, "an array pitch needs a 3-D patch");
        // the widest array of any centering: the ghosted box + 1 (side / node)
        const long long n0 = (long long)g->iupper[0] - g->ilower[0] + 2 + 2LL * g->gcw[0];
        const long long n1 = (long long)g->iupper[1] - g->ilower[1] + 2 + 2LL * g->gcw[1];
        if (g->pitch[0] < n0 || (g->pitch[1] != 0 && g->pitch[1] < n1))
            return fail(IBTK_LE_ERR_ARG, "array pitch {%d, %d} below the ghosted extent {%lld, %lld} (+1 face)",
                        g->pitch[0], g->pitch[1], n0, n1);
    }
    if (g->ndim == 3) {
        // the 3-D sweeps address one plane of an array with 32-bit byte offsets
        const long long n0 = (long long)g->iupper[0] - g->ilower[0] + 2 + 2LL * g->gcw[0];
        const long long n1 = (long long)g->iupper[1] - g->ilower[1] + 2 + 2LL * g->gcw[1];
        const long long plane = (g->pitch[0] ? g->pitch[0] : n0) * (g->pitch[1] ? g->pitch[1] : n1);
        if (8 * plane >= (1LL << 31))
            return fail(IBTK_LE_ERR_ARG, "an array plane of %lld points exceeds 2^28 (the sweeps' 32-bit offsets)",
                        plane);
    }
    return IBTK_LE_OK;
}

static bool packed(const ibtk_le_patch_geom* g) { return g->pitch[0] == 0 && g->pitch[1] == 0; }

// Strides (elements) of an array of ghosted extents n: row s1, plane s2, depth sd.
static void array_strides(const ibtk_le_patch_geom* g, const int64_t n[3], int64_t& s1, int64_t& s2, int64_t& sd) {
    if (packed(g)) {
        s1 = n[0];
        s2 = n[0] * n[1];
    } else {
        s1 = g->pitch[0];
        s2 = s1 * (g->pitch[1] ? g->pitch[1] : n[1]);
    }
    sd = s2 * n[2];
}

// Brick grid over key cells: every key whose stencil can touch any array of the
// patch (ghost box, + 1 for the shifted-frame extra face/node) gets a brick.
static int make_bin_geom(const ibtk_le_patch_geom* g, int kernel, BinGeom& bg) {
    const KernelInfo ki = kKernelInfo[kernel];
    const int B = g->ndim == 3 ? BRICK3 : BRICK2;
    std::memset(&bg, 0, sizeof(bg));
    bg.ndim = g->ndim;
    bg.shift = g->ndim == 3 ? 9 : 8;
    long long nb = 1;
    for (int d = 0; d < 3; ++d) {
        if (d >= g->ndim) {
            bg.nb[d] = 1;
            bg.nt[d] = 1;
            continue;
        }
        const int lo = g->ilower[d] - g->gcw[d];
        const int hi = g->iupper[d] + g->gcw[d] + 1;
        bg.kmin[d] = lo - ki.HI;
        const int kmax = hi - ki.LO;
        const int E = kmax - bg.kmin[d] + 1;
        const int nbd = (E + B - 1) / B;
        bg.nt[d] = (nbd + TILE - 1) / TILE;  // bricks padded to whole tiles
        bg.nb[d] = bg.nt[d] * TILE;
        nb *= bg.nb[d];
        bg.xlo[d] = g->x_lower[d];
        bg.dx[d] = g->dx[d];
        bg.ilower[d] = g->ilower[d];
    }
    const long long BV = 1LL << bg.shift;
    if ((nb + 1) * BV >= (1LL << 32))
        return fail(IBTK_LE_ERR_RANGE, "patch too large for 32-bit bin keys (%lld bricks)", nb);
    bg.nbricks = (int)nb;
    return IBTK_LE_OK;
}

// 3-D column grid over key cells: every key whose stencil can touch any array
// of the patch, for every centering (ghost box, + 1 for the extra face/node).
static int make_col_geom(const ibtk_le_patch_geom* g, int kernel, BinGeom& bg, ColGeom& cg) {
    const KernelInfo ki = kKernelInfo[kernel];
    std::memset(&bg, 0, sizeof(bg));
    std::memset(&cg, 0, sizeof(cg));
    bg.ndim = 3;
    for (int d = 0; d < 3; ++d) {
        bg.xlo[d] = g->x_lower[d];
        bg.dx[d] = g->dx[d];
        bg.ilower[d] = g->ilower[d];
        const int lo = g->ilower[d] - g->gcw[d];
        const int hi = g->iupper[d] + g->gcw[d] + 1;
        cg.org[d] = lo - ki.HI;
        cg.ext[d] = hi - ki.LO - cg.org[d] + 1;
    }
    // one empty guard column / row on each side in x and y.  The columns start
    // at the arrays' first x index + a multiple of 16: with a pitched layout
    // (ibtk_le_patch_geom::pitch) every 32-point row a sweep streams is then two
    // whole 128-byte lines.
    const int khi0 = cg.org[0] + cg.ext[0] - 1;  // last key cell in x
    const int lo0 = g->ilower[0] - g->gcw[0];
    cg.org[0] -= COLX;
    cg.org[0] -= ((cg.org[0] - lo0) % 16 + 16) % 16;
    cg.ncx = (khi0 + 1 - cg.org[0] + COLX - 1) / COLX + 1;
    cg.ncy = (cg.ext[1] + COLY - 1) / COLY + 2;
    cg.org[1] -= COLY;
    cg.ext[0] = cg.ncx * COLX;
    cg.ext[1] = cg.ncy * COLY;
    cg.nz = cg.ext[2];
    cg.ncol = cg.ncx * cg.ncy;
    if (cg.ext[0] > 65535 || cg.ext[1] > 65535)
        return fail(IBTK_LE_ERR_RANGE, "patch too wide for 16-bit packed key cells");
    const long long nb = (long long)cg.nz * cg.ncol * NBAND;
    if (nb + 1 >= (1LL << 31)) return fail(IBTK_LE_ERR_RANGE, "patch too large for 31-bit bucket keys");
    cg.nbuckets = (int)nb;
    return IBTK_LE_OK;
}

static int end_bit_for(const BinGeom& bg) {
    unsigned long long maxkey = ((unsigned long long)bg.nbricks << bg.shift);
    int bits = 1;
    while ((1ULL << bits) <= maxkey) ++bits;
    return bits;
}

// Component descriptors of a centering (LEInteractor.cpp:1017-1053 for side:
// x_lower[axis] -= dx/2 and SideGeometry::toSideBox; node: all dims shifted and
// toNodeBox; edge: every dim but `axis` shifted and toEdgeBox).
static int make_comps(const ibtk_le_patch_geom* g, int centering, int axis, double* const* q, int q_depth,
                      int Q_depth, int first, int count, Params& p) {
    const int nd = g->ndim;
    p.ncomp = count;
    for (int c = 0; c < count; ++c) {
        CompDesc& cd = p.comp[c];
        std::memset(&cd, 0, sizeof(cd));
        const int comp = first + c;  // global component index
        int shift_mask = 0, ext_mask = 0;
        double* base = nullptr;
        int depth_index = 0;
        switch (centering) {
        case IBTK_LE_CELL:
            base = q[0];
            depth_index = comp;
            cd.qcomp = comp;
            cd.axis = axis;
            break;
        case IBTK_LE_NODE:
            base = q[0];
            depth_index = comp;
            shift_mask = ext_mask = (1 << nd) - 1;
            cd.qcomp = comp;
            cd.axis = axis;
            break;
        case IBTK_LE_SIDE:
            base = q[comp];
            shift_mask = ext_mask = 1 << comp;
            cd.qcomp = comp;
            cd.axis = comp;
            break;
        case IBTK_LE_EDGE:
            base = q[comp];
            shift_mask = ext_mask = ((1 << nd) - 1) & ~(1 << comp);
            cd.qcomp = comp;
            cd.axis = comp;
            break;
        default:
            return fail(IBTK_LE_ERR_ARG, "unknown centering %d", centering);
        }
        if (!base) return fail(IBTK_LE_ERR_ARG, "null Eulerian array for component %d", comp);
        int64_t n[3] = {1, 1, 1};
        for (int d = 0; d < 3; ++d) {
            if (d < nd) {
                cd.lo[d] = g->ilower[d] - g->gcw[d];
                cd.hi[d] = g->iupper[d] + g->gcw[d] + ((ext_mask >> d) & 1);
                cd.ilower[d] = g->ilower[d];
                cd.iupper[d] = g->iupper[d];
                cd.xlo[d] = g->x_lower[d];
                if ((shift_mask >> d) & 1) cd.xlo[d] -= 0.5 * g->dx[d];
                n[d] = cd.hi[d] - cd.lo[d] + 1;
            } else {
                cd.lo[d] = cd.hi[d] = 0;
            }
        }
        cd.zcell = (nd == 3 && !((shift_mask >> 2) & 1)) ? 1 : 0;
        cd.xcell = !(shift_mask & 1) ? 1 : 0;
        cd.ycell = (nd >= 2 && !((shift_mask >> 1) & 1)) ? 1 : 0;
        int64_t sd;
        array_strides(g, n, cd.s1, cd.s2, sd);
        cd.u = base + (int64_t)depth_index * sd;
    }
    (void)q_depth;
    (void)Q_depth;
    return IBTK_LE_OK;
}

static int ncomponents(const ibtk_le_patch_geom* g, int centering, int q_depth, int Q_depth) {
    switch (centering) {
    case IBTK_LE_CELL:
    case IBTK_LE_NODE:
        if (q_depth != Q_depth)
            return -fail(IBTK_LE_ERR_DEPTH, "cell/node data: q depth %d != Q depth %d", q_depth, Q_depth);
        return q_depth;
    case IBTK_LE_SIDE:
    case IBTK_LE_EDGE:
        if (centering == IBTK_LE_EDGE && g->ndim != 3) return -fail(IBTK_LE_ERR_ARG, "edge data is 3-D only");
        if (q_depth != 1 || Q_depth != g->ndim)
            return -fail(IBTK_LE_ERR_DEPTH,
                         "side/edge-centered data requires vector-valued data (q depth 1, Q depth NDIM; got %d, %d)",
                         q_depth, Q_depth);
        return g->ndim;
    default:
        return -fail(IBTK_LE_ERR_ARG, "unknown centering %d", centering);
    }
}

static double ib6_K() { return (59.0 / 60.0) * (1.0 - std::sqrt(1.0 - (3220.0 / 3481.0))); }

// ---------------------------------------------------------------------------
// markers
// ---------------------------------------------------------------------------
extern "C" int ibtk_le_markers_create(ibtk_le_ctx ctx, ibtk_le_markers* out) {
    if (!ctx || !out) return fail(IBTK_LE_ERR_ARG, "markers_create: null argument");
    auto* m = new ibtk_le_markers_s();
    m->ctx = ctx;
    *out = m;
    return IBTK_LE_OK;
}

extern "C" int ibtk_le_markers_destroy(ibtk_le_markers m) {
    if (!m) return IBTK_LE_OK;
    hipSetDevice(m->ctx->device);
    hipStreamSynchronize(m->ctx->stream);
    for (DevBuf* b : {&m->sorted_X2, &m->xcur, &m->lvl_nbr})
        b->release();
    for (DevBuf* b : {&m->sorted_key, &m->sorted_l, &m->sorted_s, &m->sorted_X, &m->sorted_a, &m->plane_start, &m->indices,
                      &m->xshift, &m->cand_cnt, &m->cand_off, &m->cand_idx, &m->last, &m->qdst, &m->items,
                      &m->nsub, &m->isub, &m->nitems, &m->pd, &m->entry_off, &m->qin, &m->owner, &m->int_off,
                      &m->rb_cin, &m->rb_cout, &m->rb_d, &m->rb_dpre, &m->rb_mstart, &m->rb_ps2, &m->rb_mbits,
                      &m->rb_wcnt, &m->rb_wpre, &m->rb_mlist, &m->rb_scr, &m->rb_big, &m->rb_nbig, &m->cs_cnt,
                      &m->cs_off, &m->cs_pos, &m->cs_off_z, &m->zbits, &m->zst, &m->sel_gs})
        b->release();
    delete m;
    return IBTK_LE_OK;
}

extern "C" int ibtk_le_markers_count(ibtk_le_markers m) { return m ? m->n : -1; }

extern "C" int ibtk_le_markers_order(ibtk_le_markers m, const int** order_dev) {
    if (!m || !order_dev) return fail(IBTK_LE_ERR_ARG, "markers_order: null argument");
    *order_dev = m->sorted_l.as<int>();
    return IBTK_LE_OK;
}

// The 3-D sweep item table of the binned list (launch_item_table): one item per
// (column, segment), heavy ones cut into sub-segments.  No host sync: the
// sweeps launch over an upper bound of the item count and read the count on
// the device.
#ifndef IBTK_LE_STRIP
#define IBTK_LE_STRIP 1  // column rows per strip of the sweep item order (job_column)
#endif
constexpr int HEAVY_TARGET_HOST = 2048;  // le_sweep.hip HEAVY_TARGET
constexpr int LEVEL_SPLIT_TARGET = 1024;
#ifndef IBTK_LE_SPLIT_TARGET
#define IBTK_LE_SPLIT_TARGET 12288  // own markers per item above which it is cut (cfg4 items hold ~6.8K)
#endif
static int build_items(ibtk_le_ctx ctx, ibtk_le_markers m, int kernel, const int* skip_if_zero = nullptr) {
    // the candidate stream follows the bucket starts: kept only across a re-binning that
    // moved nothing since it was built (decided on the device)
    m->cs_state = (m->cs_state == 1 && skip_if_zero) ? 2 : 0;
    m->cs_skip = skip_if_zero;
    // a fresh binning's order is not the one the last re-binning's parities follow
    if (!skip_if_zero && m->zst.p) HIP_TRY(hipMemsetAsync(m->zst.p, 0, sizeof(int), ctx->stream));
    const int nj = m->npatch ? m->njobs : m->cg.ncol * m->nseg;
    // a level's items (patches of a few 32-plane segments, clustered markers on a few of
    // them) are cut at 1024 own markers, one plane per piece at least: cfg5 3.9e9 -> 4.1e9
    // (2048) -> 4.23e9 (1024; 512 and 256 are slower again, 4096 3.95e9; profiles/r04v, r04w);
    // a single patch keeps 12288 and 8 planes (cut that fine, cfg4's uniform items lose 6 %:
    // 7.04e9 -> 6.62e9, profiles/r04q, r04r)
    const int target = ctx->tune.split_target > 0 ? ctx->tune.split_target
                                                  : (m->npatch ? LEVEL_SPLIT_TARGET : IBTK_LE_SPLIT_TARGET);
    Params p;
    std::memset(&p, 0, sizeof(p));
    if (!m->npatch && ctx->zlo <= ctx->zhi) {
        // cut the items at the plane window's edges, so that the items of a
        // restricted call (ibtk_le_ctx_set_plane_window) are exactly the ones
        // next to the window's faces: the anchors reading below zlo / above zhi
        // (interp) and the planes outside [zlo, zhi] (spread)
        const KernelInfo ki = kKernelInfo[kernel];
        const int lo = ctx->zlo - m->cg.org[2], hi = ctx->zhi - m->cg.org[2];
        int c[4] = {lo - ki.LO, lo, hi - ki.HI + 1, hi + 1};
        std::sort(c, c + 4);
        for (int i = 0; i < 4; ++i)
            if (c[i] > 0 && c[i] < m->cg.nz && (p.ncut == 0 || p.cut[p.ncut - 1] != c[i])) p.cut[p.ncut++] = c[i];
    }
    // pieces per (column, segment) <= 1 + own markers / (the smaller of the two targets)
    const int tmin = std::min(target, ctx->tune.heavy_target > 0 ? ctx->tune.heavy_target : HEAVY_TARGET_HOST);
    const long long bound = (long long)nj + (long long)m->n / tmin + 1 + (long long)p.ncut * m->cg.ncol;
    if (bound * 3 >= (1LL << 31)) return fail(IBTK_LE_ERR_RANGE, "too many sweep items");
    m->item_bound = (int)bound;
    int rc;
    if ((rc = m->items.ensure(sizeof(SweepItem) * (size_t)bound))) return rc;
    if ((rc = m->nsub.ensure(2 * sizeof(int) * (size_t)std::max(nj, 1)))) return rc;
    if ((rc = m->isub.ensure(2 * sizeof(int) * (size_t)std::max(nj, 1)))) return rc;
    if ((rc = m->nitems.ensure(2 * sizeof(int)))) return rc;
    p.cg = m->cg;
    p.S = m->S;
    p.nseg = m->nseg;
    p.njobs = nj;
    p.strip = ctx->tune.strip > 0 ? ctx->tune.strip : IBTK_LE_STRIP;
    p.tune.min_piece = ctx->tune.min_piece > 0 ? ctx->tune.min_piece : (m->npatch ? 1 : 0);
    p.tune.heavy_target = ctx->tune.heavy_target;
    p.tune.heavy_min_piece = ctx->tune.heavy_min_piece;
    p.tune.heavy_first = ctx->tune.heavy_first;
    p.plane_start = m->plane_start.as<int>();
    p.items_skip = skip_if_zero;  // a re-binning where nothing moved: the table stands
    if (m->npatch) {
        p.pd = m->pd.as<PatchDesc>();
        p.npatch = m->npatch;
    }
    size_t tb = 0;
    HIP_TRY(launch_scan(nullptr, tb, m->nsub.as<int>(), m->isub.as<int>(), std::max(nj, 1), ctx->stream));
    if ((rc = ctx->temp.ensure(tb))) return rc;
    // heavy items (scheduled first): own markers per piece above 4x the mean per
    // (column, segment) pair and above 2048 -- clustered markers; uniform ones
    // never qualify
    const long long mean = (long long)m->n / std::max(nj, 1);
    int heavy = (int)std::min<long long>(std::max<long long>(4 * mean, 2048), INT_MAX / 2);
    if (ctx->tune.heavy > 0) heavy = ctx->tune.heavy;
    else if (ctx->tune.heavy < 0) heavy = INT_MAX / 2;  // off
    // a re-binning may keep the table only if it would be built the same way
    const int sig[12] = {p.ncut, p.cut[0], p.cut[1], p.cut[2], p.cut[3], p.strip, target, heavy, p.tune.min_piece,
                         p.tune.heavy_target, p.tune.heavy_min_piece, p.tune.heavy_first};
    if (std::memcmp(sig, m->items_sig, sizeof(sig)) != 0) p.items_skip = nullptr;
    std::memcpy(m->items_sig, sig, sizeof(sig));
    HIP_TRY(launch_item_table(kernel, p, target, heavy, m->nsub.as<int>(), m->isub.as<int>(),
                              m->items.as<SweepItem>(), m->nitems.as<int>(), ctx->temp.p, ctx->temp.cap, ctx->stream));
    return IBTK_LE_OK;
}

static int markers_bin_impl(ibtk_le_ctx ctx, ibtk_le_markers m, const ibtk_le_patch_geom* geom, int kernel,
                            const double* X_dev, const int* indices_dev, const double* Xshift_dev, int nindices,
                            const int* n_dev);

// The sorted entries' marker indices and positions, and the bucket starts: the
// gather records each non-empty bucket's first entry, a suffix-min scan fills in
// the empty buckets.
static int gather_buckets(ibtk_le_ctx ctx, ibtk_le_markers m, int kernel, const Params& p, int n, int nbuckets) {
    int rc;
    if ((rc = ctx->bfirst.ensure(sizeof(int) * (size_t)(nbuckets + 1)))) return rc;
    HIP_TRY(launch_gather_col(kernel, p, n, m->sorted_s.as<int>(), m->sorted_X.as<double>(), m->sorted_key.as<unsigned>(),
                              nbuckets, ctx->bfirst.as<int>(), ctx->stream));
    if ((rc = m->xcur.ensure(sizeof(double*)))) return rc;
    HIP_TRY(launch_set_xcur(m->xcur.as<double*>(), m->sorted_X.as<double>(), ctx->stream));
    m->xcur_set = true;
    size_t tb = 0;
    HIP_TRY(launch_suffix_min(nullptr, tb, ctx->bfirst.as<int>(), m->plane_start.as<int>(), nbuckets + 1, ctx->stream));
    if ((rc = ctx->temp.ensure(tb))) return rc;
    tb = ctx->temp.cap;
    HIP_TRY(launch_suffix_min(ctx->temp.p, tb, ctx->bfirst.as<int>(), m->plane_start.as<int>(), nbuckets + 1,
                              ctx->stream));
    return IBTK_LE_OK;
}

extern "C" int ibtk_le_markers_bin(ibtk_le_ctx ctx, ibtk_le_markers m, const ibtk_le_patch_geom* geom, int kernel,
                                   const double* X_dev, const int* indices_dev, const double* Xshift_dev,
                                   int nindices) {
    return markers_bin_impl(ctx, m, geom, kernel, X_dev, indices_dev, Xshift_dev, nindices, nullptr);
}

extern "C" int ibtk_le_markers_bin_count(ibtk_le_ctx ctx, ibtk_le_markers m, const ibtk_le_patch_geom* geom,
                                         int kernel, const double* X_dev, int capacity, const int* n_dev) {
    if (!n_dev) return fail(IBTK_LE_ERR_ARG, "markers_bin_count: null device count");
    if (geom && geom->ndim != 3) return fail(IBTK_LE_ERR_ARG, "markers_bin_count: 3-D patches only");
    return markers_bin_impl(ctx, m, geom, kernel, X_dev, nullptr, nullptr, capacity, n_dev);
}

// exclusive prefix sums on the context stream (rocPRIM), temp storage grown as needed
static int scan_excl(ibtk_le_ctx ctx, const int* in, int* out, int n) {
    size_t tb = 0;
    HIP_TRY(launch_scan(nullptr, tb, in, out, n, ctx->stream));
    if (int rc = ctx->temp.ensure(tb)) return rc;
    tb = ctx->temp.cap;
    HIP_TRY(launch_scan(ctx->temp.p, tb, in, out, n, ctx->stream));
    return IBTK_LE_OK;
}

// The last binning's list re-binned at new positions X_dev: the result -- sorted
// order, bucket starts, sorted positions, sweep items -- is the one
// ibtk_le_markers_bin / ibtk_le_level_bin would give for the same list at X_dev
// (the sort by (bucket, list entry) is unique), computed from the old order
// (le_sweep.hip, k_rekey .. k_rebin_scatter).  No host sync.
extern "C" int ibtk_le_markers_rebin(ibtk_le_ctx ctx, ibtk_le_markers m, const double* X_dev) {
    if (!ctx || !m) return fail(IBTK_LE_ERR_ARG, "markers_rebin: null ctx/markers");
    if (m->kernel < 0) return fail(IBTK_LE_ERR_ARG, "markers_rebin: the list was never binned");
    const int n = m->n;
    if (n > 0 && !X_dev) return fail(IBTK_LE_ERR_ARG, "null X");
    if (set_device(ctx)) return IBTK_LE_ERR_DEVICE;
    if (!m->binned3) {  // 2-D bricks: a fresh binning of the kept list
        const ibtk_le_patch_geom g = m->geom;
        return markers_bin_impl(ctx, m, &g, m->kernel, X_dev, m->has_indices ? m->indices.as<int>() : nullptr,
                                m->has_xshift ? m->xshift.as<double>() : nullptr, n, nullptr);
    }
    m->cand_valid = false;
    m->dedup_done = false;
    m->qin_valid = false;
    m->has_dups = false;
    if (n == 0) return build_items(ctx, m, m->kernel);
    const hipStream_t s = ctx->stream;
    const int nb = m->nbuckets_total;
    const int nw = (n + 31) / 32;
    int rc;
    const size_t bb = sizeof(int) * ((size_t)nb + 2), wb = sizeof(int) * ((size_t)nw + 1);
    const bool fresh = m->rb_zeroed_nb != nb || !m->rb_cin.p || m->rb_cin.cap < bb || m->rb_cout.cap < bb;
    for (DevBuf* b : {&m->rb_cin, &m->rb_cout, &m->rb_d, &m->rb_dpre, &m->rb_mstart, &m->rb_ps2, &m->rb_big})
        if ((rc = b->ensure(bb))) return rc;
    for (DevBuf* b : {&m->rb_mbits, &m->rb_wcnt, &m->rb_wpre})
        if ((rc = b->ensure(wb))) return rc;
    for (DevBuf* b : {&m->rb_mlist, &m->rb_scr})
        if ((rc = b->ensure(sizeof(int) * (size_t)n))) return rc;
    if ((rc = m->rb_nbig.ensure(sizeof(int)))) return rc;
    if ((rc = m->zbits.ensure(wb))) return rc;
    const bool znew = !m->zst.p;
    if ((rc = m->zst.ensure(2 * sizeof(int)))) return rc;
    if (znew) HIP_TRY(hipMemsetAsync(m->zst.p, 0, 2 * sizeof(int), s));
    m->rb_epoch = m->rb_epoch == INT_MAX ? 1 : m->rb_epoch + 1;  // zst[1] = 0 never matches
    if ((rc = ctx->keys_in.ensure(sizeof(unsigned) * (size_t)n))) return rc;
    if ((rc = ctx->vals_in.ensure(sizeof(int) * (size_t)n))) return rc;
    if (fresh) {  // the in/out counts start from zero (k_rebin_append leaves them so)
        HIP_TRY(hipMemsetAsync(m->rb_cin.p, 0, bb, s));
        HIP_TRY(hipMemsetAsync(m->rb_cout.p, 0, bb, s));
        m->rb_zeroed_nb = nb;
    }
    // (the sentinel word past the last and the movers' long-list queue: cleared by k_rekey)
    Params p;
    std::memset(&p, 0, sizeof(p));
    p.bg = m->bg;
    p.cg = m->cg;
    p.nbuckets_total = nb;
    p.X = X_dev;
    p.indices = m->has_indices ? m->indices.as<int>() : nullptr;
    p.Xshift = m->has_xshift ? m->xshift.as<double>() : nullptr;
    p.n_dev = m->n_dev;
    if (m->npatch) {
        p.pd = m->pd.as<PatchDesc>();
        p.npatch = m->npatch;
        p.entry_off = m->entry_off.as<int>();
    }
    RebinBufs r{};
    r.n = n;
    r.nb = nb;
    r.nw = nw;
    r.kold = m->sorted_key.as<unsigned>();
    r.lsorted = m->sorted_l.as<int>();
    r.knew = ctx->keys_in.as<unsigned>();
    r.lold = ctx->vals_in.as<int>();
    r.mbits = m->rb_mbits.as<unsigned>();
    r.wcnt = m->rb_wcnt.as<int>();
    r.wpre = m->rb_wpre.as<int>();
    r.cin = m->rb_cin.as<int>();
    r.cout = m->rb_cout.as<int>();
    r.d = m->rb_d.as<int>();
    r.dpre = m->rb_dpre.as<int>();
    r.mstart = m->rb_mstart.as<int>();
    r.mlist = m->rb_mlist.as<int>();
    r.scratch = m->rb_scr.as<int>();
    r.nbig = m->rb_nbig.as<int>();
    r.big = m->rb_big.as<int>();
    r.os = m->plane_start.as<int>();
    r.ns = m->rb_ps2.as<int>();
    r.sorted_l = m->sorted_l.as<int>();
    r.sorted_key = m->sorted_key.as<unsigned>();
    r.sorted_s = m->sorted_s.as<int>();
    if ((rc = m->sorted_X2.ensure(3 * sizeof(double) * (size_t)n))) return rc;
    if ((rc = m->xcur.ensure(sizeof(double*)))) return rc;
    if (!m->xcur_set) {
        HIP_TRY(launch_set_xcur(m->xcur.as<double*>(), m->sorted_X.as<double>(), s));
        m->xcur_set = true;
    }
    r.xcur = m->xcur.as<double*>();
    r.xa = m->sorted_X.as<double>();
    r.xb = m->sorted_X2.as<double>();
    r.order_gen = m->sel_gs.p ? m->sel_gs.as<int>() : nullptr;
    r.zbits = m->zbits.as<unsigned>();
    r.zst = m->zst.as<int>();
    r.epoch = m->rb_epoch;
    // k_rekey raises the per-bucket mover counts and k_rebin_append consumes them back
    // to zero: until the sequence has been queued whole, the next call must clear them
    m->rb_zeroed_nb = -1;
    HIP_TRY(launch_rekey(m->kernel, p, r, s));
    if ((rc = scan_excl(ctx, r.wcnt, r.wpre, nw + 1))) return rc;  // wpre[nw]: the mover count
    // everything below returns at once on the device when nothing moved
    HIP_TRY(launch_rebin_copy(m->kernel, p, r, s));
    HIP_TRY(launch_rebin_starts(r, s));
    HIP_TRY(launch_rebin_movers(r, s));
    HIP_TRY(launch_rebin_scatter(p, r, s));  // ... and the new starts into plane_start
    m->rb_zeroed_nb = nb;
    return build_items(ctx, m, m->kernel, r.wpre + nw);
}

static int markers_bin_impl(ibtk_le_ctx ctx, ibtk_le_markers m, const ibtk_le_patch_geom* geom, int kernel,
                            const double* X_dev, const int* indices_dev, const double* Xshift_dev, int nindices,
                            const int* n_dev) {
    if (!ctx || !m) return fail(IBTK_LE_ERR_ARG, "markers_bin: null ctx/markers");
    if (int rc = check_geom(geom)) return rc;
    if (kernel < 0 || kernel >= K_COUNT) return fail(IBTK_LE_ERR_UNKNOWN_KERNEL, "Unknown kernel function %d", kernel);
    if (nindices < 0) return fail(IBTK_LE_ERR_ARG, "negative list length");
    if (nindices > 0 && !X_dev) return fail(IBTK_LE_ERR_ARG, "null X");
    if (set_device(ctx)) return IBTK_LE_ERR_DEVICE;
    BinGeom bg;
    ColGeom cg{};
    const bool cols = geom->ndim == 3;
    if (cols) {
        if (int rc = make_col_geom(geom, kernel, bg, cg)) return rc;
    } else {
        if (int rc = make_bin_geom(geom, kernel, bg)) return rc;
    }
    const hipStream_t s = ctx->stream;
    const int n = nindices;
    m->n = n;
    m->kernel = kernel;
    m->ndim = geom->ndim;
    m->bg = bg;
    m->cg = cg;
    m->npatch = 0;
    m->nbuckets_total = cg.nbuckets;
    if (cols) sweep_segments(cg, m->S, m->nseg, ctx->tune.seg_items, false);
    m->geom = *geom;
    m->has_indices = indices_dev != nullptr;
    m->has_xshift = Xshift_dev != nullptr;
    m->cand_valid = false;
    m->dedup_done = false;
    m->qin_valid = false;
    m->sel_cached = false;
    m->has_dups = false;
    m->n_dev = n_dev;
    m->binned3 = cols;
    int rc = 0;
    const int B = geom->ndim == 3 ? BRICK3 : BRICK2;
    const int nplanes = cols ? cg.nbuckets : bg.nbricks * B;  // bucket starts: nplanes + 1
    if ((rc = m->plane_start.ensure(sizeof(int) * (size_t)(nplanes + 1)))) return rc;
    if (n == 0) {
        HIP_TRY(hipMemsetAsync(m->plane_start.p, 0, sizeof(int) * (size_t)(nplanes + 1), s));
        if (cols) return build_items(ctx, m, kernel);
        return IBTK_LE_OK;
    }
    if ((rc = m->sorted_key.ensure(sizeof(unsigned) * (size_t)n))) return rc;
    if ((rc = m->sorted_l.ensure(sizeof(int) * (size_t)n))) return rc;
    if ((rc = m->sorted_s.ensure(sizeof(int) * (size_t)n))) return rc;
    if ((rc = m->sorted_X.ensure(sizeof(double) * (size_t)n * geom->ndim))) return rc;
    if ((rc = ctx->keys_in.ensure(sizeof(unsigned) * (size_t)n))) return rc;
    if ((rc = ctx->vals_in.ensure(sizeof(int) * (size_t)n))) return rc;
    if (m->has_indices) {
        if ((rc = m->indices.ensure(sizeof(int) * (size_t)n))) return rc;
        if (indices_dev != m->indices.p)  // (a re-binning passes the kept list)
            HIP_TRY(hipMemcpyAsync(m->indices.p, indices_dev, sizeof(int) * (size_t)n, hipMemcpyDeviceToDevice, s));
    }
    if (m->has_xshift) {
        const size_t xb = sizeof(double) * (size_t)n * geom->ndim;
        if ((rc = m->xshift.ensure(xb))) return rc;
        if (Xshift_dev != m->xshift.p) HIP_TRY(hipMemcpyAsync(m->xshift.p, Xshift_dev, xb, hipMemcpyDeviceToDevice, s));
    }
    Params p;
    std::memset(&p, 0, sizeof(p));
    p.bg = bg;
    p.cg = cg;
    p.nbuckets_total = cg.nbuckets;
    p.X = X_dev;
    p.indices = m->has_indices ? m->indices.as<int>() : nullptr;
    p.Xshift = m->has_xshift ? m->xshift.as<double>() : nullptr;
    p.n_dev = n_dev;
    if (cols) HIP_TRY(launch_bin_col(kernel, p, n, ctx->keys_in.as<unsigned>(), ctx->vals_in.as<int>(), s));
    else HIP_TRY(launch_bin(geom->ndim, kernel, p, n, ctx->keys_in.as<unsigned>(), ctx->vals_in.as<int>(), s));
    int end_bit = 1;
    if (cols) {
        while ((1ULL << end_bit) <= (unsigned long long)cg.nbuckets) ++end_bit;
    } else {
        end_bit = end_bit_for(bg);
    }
    size_t tb = 0;
    HIP_TRY(launch_sort(nullptr, tb, ctx->keys_in.as<unsigned>(), m->sorted_key.as<unsigned>(),
                        ctx->vals_in.as<int>(), m->sorted_l.as<int>(), n, end_bit, s));
    if ((rc = ctx->temp.ensure(tb))) return rc;
    tb = ctx->temp.cap;
    HIP_TRY(launch_sort(ctx->temp.p, tb, ctx->keys_in.as<unsigned>(), m->sorted_key.as<unsigned>(),
                        ctx->vals_in.as<int>(), m->sorted_l.as<int>(), n, end_bit, s));
    p.sorted_l = m->sorted_l.as<int>();
    if (cols) {  // gather fused with the bucket starts
        if ((rc = gather_buckets(ctx, m, kernel, p, n, nplanes))) return rc;
        if (int rc2 = build_items(ctx, m, kernel)) return rc2;
    } else {
        HIP_TRY(launch_brick_start(m->sorted_key.as<unsigned>(), n, nplanes, bg.shift - (geom->ndim == 3 ? 3 : 4),
                                   m->plane_start.as<int>(), s));
        HIP_TRY(launch_gather_sorted(geom->ndim, p, n, m->sorted_s.as<int>(), m->sorted_X.as<double>(), s));
    }
    return IBTK_LE_OK;
}

// ---------------------------------------------------------------------------
// interp / spread
// ---------------------------------------------------------------------------
static bool same_geom(const ibtk_le_patch_geom& a, const ibtk_le_patch_geom& b) {
    if (a.ndim != b.ndim) return false;
    for (int d = 0; d < a.ndim; ++d) {
        if (a.ilower[d] != b.ilower[d] || a.iupper[d] != b.iupper[d] || a.gcw[d] != b.gcw[d]) return false;
        if (a.dx[d] != b.dx[d] || a.x_lower[d] != b.x_lower[d]) return false;
    }
    return true;
}

static int prepare(ibtk_le_ctx ctx, ibtk_le_markers m, int kernel, const ibtk_le_patch_geom* geom, const double* X,
                   Params& p) {
    if (!ctx || !m) return fail(IBTK_LE_ERR_ARG, "null ctx/markers");
    if (int rc = check_geom(geom)) return rc;
    if (kernel < 0 || kernel >= K_COUNT) return fail(IBTK_LE_ERR_UNKNOWN_KERNEL, "Unknown kernel function %d", kernel);
    if (m->kernel != kernel)
        return fail(IBTK_LE_ERR_ARG, "markers were binned for kernel %s, not %s",
                    m->kernel >= 0 ? kNames[m->kernel] : "(none)", kNames[kernel]);
    if (m->npatch) return fail(IBTK_LE_ERR_ARG, "markers were binned for a level: use ibtk_le_level_interp/spread");
    if (!same_geom(m->geom, *geom)) return fail(IBTK_LE_ERR_ARG, "markers were binned for a different patch geometry");
    if (m->n > 0 && !X) return fail(IBTK_LE_ERR_ARG, "null X");
    std::memset(&p, 0, sizeof(p));
    p.bg = m->bg;
    p.cg = m->cg;
    p.S = m->S;
    p.nseg = m->nseg;
    p.items = m->items.as<SweepItem>();
    p.nitems = m->nitems.as<int>();
    p.item_bound = m->item_bound;
    p.nbuckets_total = m->nbuckets_total;
    p.sorted_a = m->sorted_a.as<unsigned>();
    p.nsorted = m->n;
    p.X = X;
    p.indices = m->has_indices ? m->indices.as<int>() : nullptr;
    p.Xshift = m->has_xshift ? m->xshift.as<double>() : nullptr;
    p.sorted_l = m->sorted_l.as<int>();
    p.sorted_s = m->sorted_s.as<int>();
    p.sorted_X = m->sorted_X.as<double>();
    p.sorted_X_ref = m->xcur_set ? m->xcur.as<double*>() : nullptr;
    p.sorted_key = m->sorted_key.as<unsigned>();
    p.plane_start = m->plane_start.as<int>();
    p.err = ctx->err.as<int>();
    p.sink = ctx->sink.as<double>();
    p.tune = ctx->tune;
    p.zmode = ctx->zmode;
    p.zlo = ctx->zlo;
    p.zhi = ctx->zhi;
    p.K6 = ib6_K();
    p.h3 = geom->ndim == 3 ? (geom->dx[0] * geom->dx[1]) * geom->dx[2] : geom->dx[0] * geom->dx[1];
    return IBTK_LE_OK;
}

// A list that names a marker more than once (LIndexSetData's ghost-box list holds
// periodic images) writes V(:,s) from its last entry, as the Fortran's
// sequential l-loop does.  Built once per binning, on the first interp after it
// (two host syncs; identity lists skip it).
static int build_dedup(ibtk_le_ctx ctx, ibtk_le_markers m) {
    if (m->dedup_done) return IBTK_LE_OK;
    m->dedup_done = true;
    m->has_dups = false;
    if (!m->has_indices || m->n <= 1) return IBTK_LE_OK;
    const hipStream_t s = ctx->stream;
    int rc;
    if ((rc = ctx->counts.ensure(2 * sizeof(int)))) return rc;
    int* dv = ctx->counts.as<int>();
    HIP_TRY(hipMemsetAsync(dv, 0xff, sizeof(int), s));
    HIP_TRY(hipMemsetAsync(dv + 1, 0, sizeof(int), s));
    HIP_TRY(launch_max_index(m->indices.as<int>(), m->n, dv, s));
    int mx = -1;
    HIP_TRY(hipMemcpyAsync(&mx, dv, sizeof(int), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (mx < 0) return fail(IBTK_LE_ERR_ARG, "negative marker index in the list");
    if ((rc = m->last.ensure(sizeof(int) * ((size_t)mx + 1)))) return rc;
    if ((rc = m->qdst.ensure(sizeof(int) * (size_t)m->n))) return rc;
    HIP_TRY(hipMemsetAsync(m->last.p, 0xff, sizeof(int) * ((size_t)mx + 1), s));
    HIP_TRY(launch_dedup(m->indices.as<int>(), m->sorted_l.as<int>(), m->sorted_s.as<int>(), m->n, m->last.as<int>(),
                         m->qdst.as<int>(), dv + 1, s));
    int ndup = 0;
    HIP_TRY(hipMemcpyAsync(&ndup, dv + 1, sizeof(int), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    m->has_dups = ndup > 0;
    return IBTK_LE_OK;
}

// Counted spread sweeps (ibtk_le_ctx_count_adds): the ds_add_f64 the sweep issues,
// for the LDS-atomic bound (bench.py's roofline.lds_atomic).  One host sync per
// launch, so only outside timed regions.
static int adds_begin(ibtk_le_ctx ctx, Params& p, bool reset) {
    p.nadd = nullptr;
    if (!ctx->count_adds) return IBTK_LE_OK;
    if (int rc = ctx->adds.ensure(2 * sizeof(unsigned long long))) return rc;
    HIP_TRY(hipMemsetAsync(ctx->adds.p, 0, 2 * sizeof(unsigned long long), ctx->stream));
    if (reset) ctx->last_adds[0] = ctx->last_adds[1] = 0;
    p.nadd = ctx->adds.as<unsigned long long>();
    return IBTK_LE_OK;
}
static int adds_end(ibtk_le_ctx ctx, Params& p) {
    if (!p.nadd) return IBTK_LE_OK;
    unsigned long long h[2] = {0, 0};
    HIP_TRY(hipMemcpyAsync(h, p.nadd, sizeof(h), hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    ctx->last_adds[0] += h[0];
    ctx->last_adds[1] += h[1];
    p.nadd = nullptr;
    return IBTK_LE_OK;
}

extern "C" int ibtk_le_ctx_count_adds(ibtk_le_ctx ctx, int enable) {
    if (!ctx) return fail(IBTK_LE_ERR_ARG, "null ctx");
    ctx->count_adds = enable != 0;
    return IBTK_LE_OK;
}

extern "C" int ibtk_le_ctx_last_adds(ibtk_le_ctx ctx, unsigned long long* out) {
    if (!ctx || !out) return fail(IBTK_LE_ERR_ARG, "null argument");
    out[0] = ctx->last_adds[0];
    out[1] = ctx->last_adds[1];
    return IBTK_LE_OK;
}

// Diagnostic phase clocks of the spread sweep (IBTK_LE_STAMPS=1 with a
// -DIBTK_LE_CLOCKS=1 build): per-item cycle totals, summarised on stderr.
static int stamps_begin(ibtk_le_ctx ctx, size_t nst, Params& p) {
    if (!ctx->stamps_on) return IBTK_LE_OK;
    if (int rc = ctx->stamps.ensure(nst * sizeof(unsigned long long))) return rc;
    HIP_TRY(hipMemsetAsync(ctx->stamps.p, 0, nst * sizeof(unsigned long long), ctx->stream));
    p.stamps = ctx->stamps.as<unsigned long long>();
    return IBTK_LE_OK;
}
static int stamps_report(ibtk_le_ctx ctx, size_t nst, Params& p) {
    if (!p.stamps) return IBTK_LE_OK;
    std::vector<unsigned long long> h(nst);
    HIP_TRY(hipMemcpyAsync(h.data(), p.stamps, nst * sizeof(unsigned long long), hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    double tot[6] = {0, 0, 0, 0, 0, 0};
    long items = 0;
    std::vector<unsigned long long> sums;
    for (size_t i = 0; i < nst / 8; ++i) {
        unsigned long long sum = 0;
        for (int k = 0; k < 6; ++k) sum += h[i * 8 + k];
        if (!sum) continue;
        ++items;
        sums.push_back(sum);
        for (int k = 0; k < 6; ++k) tot[k] += (double)h[i * 8 + k];
    }
    std::sort(sums.begin(), sums.end());
    const double q99 = sums.empty() ? 0.0 : (double)sums[(size_t)(0.99 * (sums.size() - 1))];
    const double mx = sums.empty() ? 0.0 : (double)sums.back();
    double all = 0.0;
    for (unsigned long long v : sums) all += (double)v;
    const long n = items > 0 ? items : 1;
    fprintf(stderr,
            "spread stamps: %ld items; mean cycles/item: prologue %.0f writeback+put %.0f prefetch+deal+weights %.0f "
            "adds %.0f rest %.0f epilogue %.0f; item total mean %.0f p99 %.0f max %.0f; sum over items %.3e\n",
            items, tot[0] / n, tot[1] / n, tot[2] / n, tot[3] / n, tot[4] / n, tot[5] / n, all / n, q99, mx, all);
    p.stamps = nullptr;
    return IBTK_LE_OK;
}

int ibtk_le::interp_impl(ibtk_le_ctx ctx, ibtk_le_markers m, int kernel, int centering, int axis, const void* geomv,
                         const double* const* q_dev, int q_depth, double* Q_dev, int Q_depth, const double* X_dev,
                         bool check_ghosts, const int* iper) {
    const ibtk_le_patch_geom* geom = static_cast<const ibtk_le_patch_geom*>(geomv);
    Params p;
    if (int rc = prepare(ctx, m, kernel, geom, X_dev, p)) return rc;
    if (iper)
        for (int d = 0; d < 3; ++d) p.iper[d] = iper[d] ? 1 : 0;
    // LEInteractor.cpp:2416-2426: interp needs min(gcw) >= floor(stencil/2)+1
    int gmin = geom->gcw[0];
    for (int d = 1; d < geom->ndim; ++d) gmin = std::min(gmin, geom->gcw[d]);
    if (check_ghosts && gmin < ibtk_le_min_ghost_width(kernel))
        return fail(IBTK_LE_ERR_GHOST_WIDTH,
                    "LEInteractor::interpolate(): insufficient ghost cells: kernel %s needs %d, ghost width %d",
                    kNames[kernel], ibtk_le_min_ghost_width(kernel), gmin);
    const int nc = ncomponents(geom, centering, q_depth, Q_depth);
    if (nc < 0) return -nc;
    if (m->n == 0) return IBTK_LE_OK;  // LEInteractor.cpp:2427
    if (!Q_dev || !q_dev) return fail(IBTK_LE_ERR_ARG, "null Q or q");
    if (set_device(ctx)) return IBTK_LE_ERR_DEVICE;
    if (int rc = build_dedup(ctx, m)) return rc;
    p.qdst = m->has_dups ? m->qdst.as<int>() : nullptr;
    p.Qout = Q_dev;
    p.Q_depth = Q_depth;
    ctx->ev_valid = false;
    for (int first = 0; first < nc; first += MAXC) {
        const int cnt = std::min(MAXC, nc - first);
        if (int rc = make_comps(geom, centering, axis, const_cast<double* const*>(q_dev), q_depth, Q_depth, first,
                                cnt, p))
            return rc;
        const bool t = ctx->timing && first == 0;
        if (geom->ndim == 3)
            HIP_TRY(launch_interp_sweep(kernel, p, m->n, ctx->stream, t ? ctx->ev0 : nullptr, t ? ctx->ev1 : nullptr));
        else
            HIP_TRY(launch_interp(geom->ndim, kernel, p, m->n, ctx->stream, t ? ctx->ev0 : nullptr,
                                  t ? ctx->ev1 : nullptr));
        if (t) ctx->ev_valid = true;
    }
    return IBTK_LE_OK;
}

extern "C" int ibtk_le_interp(ibtk_le_ctx ctx, ibtk_le_markers m, int kernel, int centering, int axis,
                              const ibtk_le_patch_geom* geom, const double* const* q_dev, int q_depth, double* Q_dev,
                              int Q_depth, const double* X_dev) {
    return ibtk_le::interp_impl(ctx, m, kernel, centering, axis, geom, q_dev, q_depth, Q_dev, Q_depth, X_dev, true);
}

// ibtk_le_fill_periodic_ghosts + ibtk_le_interp: the 3-D column sweep reads every ghost
// point of the ghost box at its periodic image (the value the fill copies there) and
// writes no ghost; other binnings: the two calls
extern "C" int ibtk_le_fill_interp(ibtk_le_ctx ctx, ibtk_le_markers m, int kernel, int centering, int axis,
                                   const ibtk_le_patch_geom* geom, const double* const* q_dev, int q_depth,
                                   double* Q_dev, int Q_depth, const double* X_dev, const int* periodic) {
    int per[3] = {1, 1, 1};
    if (periodic)
        for (int d = 0; d < 3; ++d) per[d] = (geom && d < geom->ndim) ? (periodic[d] ? 1 : 0) : 0;
    if (!geom || geom->ndim != 3 || !m || !m->binned3) {
        if (int rc = ibtk_le_fill_periodic_ghosts(ctx, geom, centering, const_cast<double* const*>(q_dev), q_depth, per))
            return rc;
        return ibtk_le::interp_impl(ctx, m, kernel, centering, axis, geom, q_dev, q_depth, Q_dev, Q_depth, X_dev, true);
    }
    // the fill's own argument check (ghost_op), so that the fused form fails where the pair does
    for (int d = 0; d < 3; ++d)
        if (per[d] && geom->iupper[d] - geom->ilower[d] + 1 < 2 * geom->gcw[d] + 1)
            return fail(IBTK_LE_ERR_ARG, "periodic dim %d narrower than 2*ghost+1", d);
    return ibtk_le::interp_impl(ctx, m, kernel, centering, axis, geom, q_dev, q_depth, Q_dev, Q_depth, X_dev, true, per);
}

// Super-brick candidate lists (k_cand): count, exclusive scan, write.  Built once
// per binning, on the first spread after it.
static int build_candidates(ibtk_le_ctx ctx, ibtk_le_markers m, const Params& p) {
    if (m->cand_valid) return IBTK_LE_OK;
    const hipStream_t s = ctx->stream;
    const int items = m->bg.nbricks / (m->ndim == 3 ? 8 : 4) * cand_classes(m->ndim, m->kernel);
    int rc = 0;
    if ((rc = m->cand_cnt.ensure(sizeof(int) * (size_t)(items + 1)))) return rc;
    if ((rc = m->cand_off.ensure(sizeof(int) * (size_t)(items + 1)))) return rc;
    if ((rc = m->cand_idx.ensure(sizeof(int) * (size_t)m->n * (m->ndim == 3 ? 8 : 4)))) return rc;
    HIP_TRY(hipMemsetAsync(m->cand_cnt.p, 0, sizeof(int) * (size_t)(items + 1), s));
    HIP_TRY(launch_cand(m->ndim, m->kernel, p, false, m->cand_cnt.as<int>(), nullptr, s));
    size_t tb = 0;
    HIP_TRY(launch_scan(nullptr, tb, m->cand_cnt.as<int>(), m->cand_off.as<int>(), items + 1, s));
    if ((rc = ctx->temp.ensure(tb))) return rc;
    tb = ctx->temp.cap;
    HIP_TRY(launch_scan(ctx->temp.p, tb, m->cand_cnt.as<int>(), m->cand_off.as<int>(), items + 1, s));
    HIP_TRY(launch_cand(m->ndim, m->kernel, p, true, m->cand_off.as<int>(), m->cand_idx.as<int>(), s));
    m->cand_valid = true;
    return IBTK_LE_OK;
}

// The 3-D spread's F gather (sorted_F from Q and sorted_s, both ready on `stream`) does not
// depend on the candidate stream, whose rebuild after a re-binning (k_cand_count, the scan,
// k_cand_write: about 1 ms at cfg4) leaves CUs idle: when the stream is rebuilt, the
// gather runs beside it on the side stream (cfg4 moving: spread 14.6 -> 14.4 ms a step,
// profiles/r06/side_gather_ab.txt); a standing stream keeps the gather in line.  The fork orders the gather after everything on `stream` so far (the
// binning, the previous sweep still reading sorted_F); the join orders the sweep after it.
// Worth its cross-stream hops (about 0.05 ms a step) only on a large gather: cfg4 (1e8
// markers) gains 0.2 ms, cfg5 (1e7, a level) loses 0.04 ms; the gain scales with n, even
// at about 2.5e7.  side_gather: 0 auto (n >= 2^25), 1 always, -1 never.
static bool side_gather(ibtk_le_ctx ctx, ibtk_le_markers m) {
    const int t = ctx->tune.side_gather;
    return t > 0 || (t == 0 && m->n >= (1 << 25));
}
static int gather_fork(ibtk_le_ctx ctx, const Params& p) {
    if (!ctx->side) {  // created together, or not at all
        if (!ctx->ev_fork) HIP_TRY(hipEventCreateWithFlags(&ctx->ev_fork, hipEventDisableTiming));
        if (!ctx->ev_join) HIP_TRY(hipEventCreateWithFlags(&ctx->ev_join, hipEventDisableTiming));
        hipStream_t st = nullptr;
        HIP_TRY(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
        ctx->side = st;
    }
    HIP_TRY(hipEventRecord(ctx->ev_fork, ctx->stream));
    HIP_TRY(hipStreamWaitEvent(ctx->side, ctx->ev_fork, 0));
    HIP_TRY(launch_gather_F(p, ctx->side));
    HIP_TRY(hipEventRecord(ctx->ev_join, ctx->side));
    return IBTK_LE_OK;
}
static int gather_join(ibtk_le_ctx ctx) {
    HIP_TRY(hipStreamWaitEvent(ctx->stream, ctx->ev_join, 0));
    return IBTK_LE_OK;
}

static int spread_impl(ibtk_le_ctx ctx, ibtk_le_markers m, int kernel, int centering, int axis,
                       const ibtk_le_patch_geom* geom, double* const* q_dev, int q_depth, const double* Q_dev,
                       int Q_depth, const double* ds_dev, const double* X_dev, bool zero_ghosts = false,
                       bool zero_first = false);

extern "C" int ibtk_le_spread(ibtk_le_ctx ctx, ibtk_le_markers m, int kernel, int centering, int axis,
                              const ibtk_le_patch_geom* geom, double* const* q_dev, int q_depth, const double* Q_dev,
                              int Q_depth, const double* X_dev) {
    return spread_impl(ctx, m, kernel, centering, axis, geom, q_dev, q_depth, Q_dev, Q_depth, nullptr, X_dev);
}

// ibtk_le_zero_ghosts + ibtk_le_spread: the 3-D column sweeps start the owned ghost
// points from 0 (no separate pass over the ghost layers); 2-D: the two calls
extern "C" int ibtk_le_zero_ghosts_spread(ibtk_le_ctx ctx, ibtk_le_markers m, int kernel, int centering, int axis,
                                          const ibtk_le_patch_geom* geom, double* const* q_dev, int q_depth,
                                          const double* Q_dev, int Q_depth, const double* X_dev) {
    if (!geom || geom->ndim != 3 || !m || m->n == 0 || !m->binned3) {
        if (int rc = ibtk_le_zero_ghosts(ctx, geom, centering, q_dev, q_depth)) return rc;
        return spread_impl(ctx, m, kernel, centering, axis, geom, q_dev, q_depth, Q_dev, Q_depth, nullptr, X_dev);
    }
    return spread_impl(ctx, m, kernel, centering, axis, geom, q_dev, q_depth, Q_dev, Q_depth, nullptr, X_dev, true);
}

// Every point of the component arrays to 0 (a pitched layout: the whole span, row
// padding included), on the context stream
static int zero_comps(ibtk_le_ctx ctx, const ibtk_le_patch_geom* geom, int centering, int axis, double* const* q_dev,
                      int q_depth, int Q_depth) {
    if (int rc = check_geom(geom)) return rc;
    if (!q_dev) return fail(IBTK_LE_ERR_ARG, "null q");
    const int nc = ncomponents(geom, centering, q_depth, Q_depth);
    if (nc < 0) return -nc;
    if (set_device(ctx)) return IBTK_LE_ERR_DEVICE;
    Params p;
    for (int first = 0; first < nc; first += MAXC) {
        const int cnt = std::min(MAXC, nc - first);
        if (int rc = make_comps(geom, centering, axis, q_dev, q_depth, Q_depth, first, cnt, p)) return rc;
        for (int c = 0; c < cnt; ++c) {
            const CompDesc& cd = p.comp[c];
            const size_t pts = (size_t)cd.s2 * (size_t)(cd.hi[2] - cd.lo[2] + 1);
            HIP_TRY(hipMemsetAsync(cd.u, 0, sizeof(double) * pts, ctx->stream));
        }
    }
    return IBTK_LE_OK;
}

// LDataManager::spread's target: the whole of f set to 0, ghosts included
// (LDataManager.cpp:596, setToScalar(f, 0, interior_only = false)), then
// LEInteractor::spread into it (:625-660).  A 3-D column binning does both in the
// spread's sweep: its items start every owned point from 0 instead of reading it and
// items no marker reaches store the zeros, so f is written once and never read.
// Other binnings: the zeroing, then ibtk_le_spread.
extern "C" int ibtk_le_zero_spread(ibtk_le_ctx ctx, ibtk_le_markers m, int kernel, int centering, int axis,
                                   const ibtk_le_patch_geom* geom, double* const* q_dev, int q_depth,
                                   const double* Q_dev, int Q_depth, const double* X_dev) {
    if (!ctx || !m) return fail(IBTK_LE_ERR_ARG, "zero_spread: null ctx/markers");
    if (!geom || geom->ndim != 3 || !m || m->n == 0 || !m->binned3) {
        if (int rc = zero_comps(ctx, geom, centering, axis, q_dev, q_depth, Q_depth)) return rc;
        return spread_impl(ctx, m, kernel, centering, axis, geom, q_dev, q_depth, Q_dev, Q_depth, nullptr, X_dev);
    }
    return spread_impl(ctx, m, kernel, centering, axis, geom, q_dev, q_depth, Q_dev, Q_depth, nullptr, X_dev, false,
                       true);
}

extern "C" int ibtk_le_spread_ds(ibtk_le_ctx ctx, ibtk_le_markers m, int kernel, int centering, int axis,
                                 const ibtk_le_patch_geom* geom, double* const* q_dev, int q_depth,
                                 const double* Q_dev, int Q_depth, const double* ds_dev, const double* X_dev) {
    if (!ds_dev && m && m->n > 0) return fail(IBTK_LE_ERR_ARG, "null ds");
    return spread_impl(ctx, m, kernel, centering, axis, geom, q_dev, q_depth, Q_dev, Q_depth, ds_dev, X_dev);
}

// ---------------------------------------------------------------------------
// USER_DEFINED kernel function: LEInteractor::userDefinedInterpolate / Spread
// (LEInteractor.cpp:3141-3266, 3268-3393, dispatched at :2688 and :3007).  The
// kernel function is a host function pointer, so the host evaluates it: the
// list's positions come back from the device once, the host forms every entry's
// clipped stencil and weights per component frame, and the device sums (interp:
// one lane per entry, the reference's loop order; spread: contributions keyed by
// grid point, stably sorted and summed point by point in list order -- the
// sequential l-loop's order, so the result is the reference arithmetic's and
// bit-stable).  One host synchronization per call.
// ---------------------------------------------------------------------------
static int user_call(ibtk_le_ctx ctx, bool spread, int centering, int axis, const ibtk_le_patch_geom* geom,
                     double* const* q_dev, int q_depth, double* Q_dev, int Q_depth, const double* X_dev,
                     const int* indices_dev, const double* Xshift_dev, int n) {
    if (!ctx) return fail(IBTK_LE_ERR_ARG, "null ctx");
    if (int rc = check_geom(geom)) return rc;
    if (n < 0) return fail(IBTK_LE_ERR_ARG, "negative list length");
    const int nd = geom->ndim;
    const int S = g_user_size;
    int gmin = geom->gcw[0];
    for (int d = 1; d < nd; ++d) gmin = std::min(gmin, geom->gcw[d]);
    if (!spread && gmin < S / 2 + 1)  // LEInteractor.cpp:2416-2426
        return fail(IBTK_LE_ERR_GHOST_WIDTH,
                    "LEInteractor::interpolate(): insufficient ghost cells: kernel USER_DEFINED needs %d, ghost width %d",
                    S / 2 + 1, gmin);
    const int nc = ncomponents(geom, centering, q_depth, Q_depth);
    if (nc < 0) return -nc;
    if (n == 0) return IBTK_LE_OK;
    if (!X_dev || !Q_dev || !q_dev) return fail(IBTK_LE_ERR_ARG, "null X, Q or q");
    if (set_device(ctx)) return IBTK_LE_ERR_DEVICE;
    const hipStream_t st = ctx->stream;
    int rc;
    if ((rc = ctx->usr_x0.ensure(sizeof(double) * (size_t)n * nd)) || (rc = ctx->usr_x1.ensure(sizeof(double) * (size_t)n * nd)) ||
        (rc = ctx->usr_s.ensure(sizeof(int) * (size_t)n)))
        return rc;
    HIP_TRY(launch_user_gather(X_dev, indices_dev, Xshift_dev, n, nd, ctx->usr_x0.as<double>(), ctx->usr_x1.as<double>(),
                               ctx->usr_s.as<int>(), st));
    std::vector<double> Xr((size_t)n * nd), Xs((size_t)n * nd);
    std::vector<int> sidx((size_t)n);
    HIP_TRY(hipMemcpyAsync(Xr.data(), ctx->usr_x0.p, sizeof(double) * Xr.size(), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(Xs.data(), ctx->usr_x1.p, sizeof(double) * Xs.size(), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(sidx.data(), ctx->usr_s.p, sizeof(int) * sidx.size(), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    std::vector<int> last;
    if (!spread) {  // the last entry naming each marker writes its Q
        last.assign((size_t)n, 0);
        std::unordered_map<int, int> at;
        at.reserve((size_t)n * 2);
        for (int l = 0; l < n; ++l) at[sidx[l]] = l;
        for (const auto& kv : at) last[kv.second] = 1;
        if ((rc = ctx->usr_last.ensure(sizeof(int) * (size_t)n))) return rc;
        HIP_TRY(hipMemcpyAsync(ctx->usr_last.p, last.data(), sizeof(int) * (size_t)n, hipMemcpyHostToDevice, st));
    }
    if ((rc = ctx->usr_lo.ensure(sizeof(int) * (size_t)n * 3)) || (rc = ctx->usr_cnt.ensure(sizeof(int) * (size_t)n * 3)) ||
        (rc = ctx->usr_w.ensure(sizeof(double) * (size_t)n * 3 * S)))
        return rc;
    std::vector<int> lo((size_t)n * 3, 0), cnt((size_t)n * 3, 1);
    std::vector<double> w((size_t)n * 3 * S, 0.0);
    for (int c = 0; c < nc; ++c) {
        Params p;
        std::memset(&p, 0, sizeof(p));
        if ((rc = make_comps(geom, centering, axis, q_dev, q_depth, Q_depth, c, 1, p))) return rc;
        const CompDesc& cd = p.comp[0];
        if (spread) {
            int64_t vol = 1;
            for (int d = 0; d < nd; ++d) vol *= (int64_t)(cd.hi[d] - cd.lo[d] + 1);
            const int64_t span = (int64_t)(cd.hi[0] - cd.lo[0]) + (nd > 1 ? (int64_t)(cd.hi[1] - cd.lo[1]) * cd.s1 : 0) +
                                 (nd > 2 ? (int64_t)(cd.hi[2] - cd.lo[2]) * cd.s2 : 0);
            if (span >= 0xffffffffLL || (int64_t)n * S * S * (nd == 3 ? S : 1) >= (1LL << 31))
                return fail(IBTK_LE_ERR_RANGE, "USER_DEFINED spread: array or list too large for 32-bit keys");
            (void)vol;
        }
        // userDefinedInterpolate/Spread's stencil and weights (LEInteractor.cpp:3169-3239)
        for (int l = 0; l < n; ++l) {
            for (int d = 0; d < nd; ++d) {
                const double x = Xs[(size_t)nd * l + d];         // X + X_shift
                const double xraw = Xr[(size_t)nd * l + d];      // X alone (the even-stencil test, :3188)
                const int center = static_cast<int>(std::floor((x - cd.xlo[d]) / geom->dx[d])) + cd.ilower[d];
                const double xcell = cd.xlo[d] + (static_cast<double>(center - cd.ilower[d]) + 0.5) * geom->dx[d];
                int sl, su;
                if (S % 2 == 0) {
                    if (xraw < xcell) {
                        sl = center - S / 2;
                        su = center + S / 2 - 1;
                    } else {
                        sl = center - S / 2 + 1;
                        su = center + S / 2;
                    }
                } else {
                    sl = center - S / 2;
                    su = center + S / 2;
                }
                sl = std::min(std::max(sl, cd.lo[d]), cd.hi[d]);  // :3209-3213
                su = std::min(std::max(su, cd.lo[d]), cd.hi[d]);
                lo[3 * (size_t)l + d] = sl;
                cnt[3 * (size_t)l + d] = su - sl + 1;
                double* wl = &w[((size_t)3 * l + d) * S];
                for (int ic = sl; ic <= su; ++ic)
                    wl[ic - sl] = g_user_fcn((x - (xcell + static_cast<double>(ic - center) * geom->dx[d])) / geom->dx[d]);
            }
        }
        HIP_TRY(hipMemcpyAsync(ctx->usr_lo.p, lo.data(), sizeof(int) * lo.size(), hipMemcpyHostToDevice, st));
        HIP_TRY(hipMemcpyAsync(ctx->usr_cnt.p, cnt.data(), sizeof(int) * cnt.size(), hipMemcpyHostToDevice, st));
        HIP_TRY(hipMemcpyAsync(ctx->usr_w.p, w.data(), sizeof(double) * w.size(), hipMemcpyHostToDevice, st));
        UserDesc u;
        std::memset(&u, 0, sizeof(u));
        u.cd = cd;
        u.ndim = nd;
        u.S = S;
        u.n = n;
        u.lo = ctx->usr_lo.as<int>();
        u.cnt = ctx->usr_cnt.as<int>();
        u.w = ctx->usr_w.as<double>();
        u.sidx = ctx->usr_s.as<int>();
        u.last = ctx->usr_last.as<int>();
        u.Q = Q_dev;
        u.Qout = Q_dev;
        u.Q_depth = Q_depth;
        u.dxprod = nd == 3 ? (geom->dx[0] * geom->dx[1]) * geom->dx[2] : geom->dx[0] * geom->dx[1];
        if (!spread) {
            HIP_TRY(launch_user_interp(u, st));
        } else {
            const int per = nd == 3 ? S * S * S : S * S;
            const int ncon = n * per;
            if ((rc = ctx->keys_in.ensure(sizeof(unsigned) * 2 * (size_t)ncon)) ||
                (rc = ctx->vals_in.ensure(sizeof(int) * 2 * (size_t)ncon)) ||
                (rc = ctx->fbuf.ensure(sizeof(double) * (size_t)ncon)))
                return rc;
            unsigned* k0 = ctx->keys_in.as<unsigned>();
            int* v0 = ctx->vals_in.as<int>();
            HIP_TRY(launch_user_contrib(u, k0, v0, ctx->fbuf.as<double>(), st));
            size_t tb = 0;
            HIP_TRY(launch_sort(nullptr, tb, k0, k0 + ncon, v0, v0 + ncon, ncon, 32, st));
            if ((rc = ctx->temp.ensure(tb))) return rc;
            tb = ctx->temp.cap;
            HIP_TRY(launch_sort(ctx->temp.p, tb, k0, k0 + ncon, v0, v0 + ncon, ncon, 32, st));
            HIP_TRY(launch_user_segsum(u, k0 + ncon, v0 + ncon, ctx->fbuf.as<double>(), ncon, st));
        }
        // the host tables are reused by the next component: wait for the uploads
        HIP_TRY(hipStreamSynchronize(st));
    }
    return IBTK_LE_OK;
}

extern "C" int ibtk_le_user_interp(ibtk_le_ctx ctx, int centering, int axis, const ibtk_le_patch_geom* geom,
                                   const double* const* q_dev, int q_depth, double* Q_dev, int Q_depth,
                                   const double* X_dev, const int* indices_dev, const double* Xshift_dev, int n) {
    return user_call(ctx, false, centering, axis, geom, const_cast<double* const*>(q_dev), q_depth, Q_dev, Q_depth, X_dev,
                     indices_dev, Xshift_dev, n);
}
extern "C" int ibtk_le_user_spread(ibtk_le_ctx ctx, int centering, int axis, const ibtk_le_patch_geom* geom,
                                   double* const* q_dev, int q_depth, const double* Q_dev, int Q_depth,
                                   const double* X_dev, const int* indices_dev, const double* Xshift_dev, int n) {
    return user_call(ctx, true, centering, axis, geom, q_dev, q_depth, const_cast<double*>(Q_dev), Q_depth, X_dev,
                     indices_dev, Xshift_dev, n);
}

// The 3-D spread's candidate stream of m's binning (le_sweep.hip, launch_cand_stream):
// built on the first spread after a binning, kept until the next; p.cs_* set.  A
// closed-form kernel's components in a z frame shifted by -dz/2 (p.comp) need it split by
// their anchor (cs_off_z): a stream built without the split is rebuilt with it, and one
// built with it stands across a re-binning only if that moved no marker and changed no
// shifted-z anchor (positions move within their cells).
// A closed-form kernel's stream is always split by the shifted-z anchor, whichever
// components a call spreads: the order of a column-anchor's candidates -- the order in
// which they add into a point -- then depends on the binning alone, not on which
// centerings were spread since it (advisor, round 5)
static bool cand_split(int k) { return k == K_IB_4 || k == K_BSPLINE_4 || k == K_IB_6 || k == K_IB_4_W8; }
// the stream stands as built: cand_stream launches nothing
static bool cand_stream_built(ibtk_le_markers m) {
    return m->cs_state == 1 && m->cs_pos.p && (m->cs_split || !cand_split(m->kernel));
}
static int cand_stream(ibtk_le_ctx ctx, ibtk_le_markers m, Params& p) {
    const long long ncl = (long long)m->nbuckets_total / NBAND;
    const long long nclz = m->npatch ? m->nclz : (long long)m->cg.ncol * (m->cg.nz + 1);
    const int k = m->kernel;
    const bool split = cand_split(k);
    // A marker is a candidate of at most four columns (its own, one x- and one y-neighbour,
    // the corner between them: a stencil never reaches both neighbours in a dim), so 4 n
    // positions always hold the stream (16 bytes a marker; about 1.3 of the 4 are used by
    // uniform IB_4 markers).  Offsets are 32-bit: a stream of 2^31 entries or more raises
    // device flag 16 (k_cand_write checks its 64-bit length) instead of being refused here.
    const long long cap = std::min(std::max(4LL * m->n, 1LL), (1LL << 31) - 1);
    if (ncl + 1 >= (1LL << 31) || nclz + 1 >= (1LL << 31))
        return fail(IBTK_LE_ERR_RANGE, "candidate stream too long");
    p.cs_off = m->cs_off.as<int>();
    p.cs_pos = m->cs_pos.as<int>();
    p.cs_total = (int)cap;
    p.cs_off_z = m->cs_split ? m->cs_off_z.as<int>() : nullptr;
    p.cs_rint = k == K_IB_4 ? 1 : 0;  // the IB_4 spread anchors by rint (spread_setup)
    if (cand_stream_built(m)) return IBTK_LE_OK;
    int rc;
    // cs_cnt: ncl + 1 counts, then the stream's 64-bit length (8-byte aligned)
    const size_t tot_at = (sizeof(int) * (size_t)(ncl + 1) + 7) / 8 * 8;
    if ((rc = m->cs_cnt.ensure(tot_at + sizeof(unsigned long long)))) return rc;
    if ((rc = m->cs_off.ensure(sizeof(int) * (size_t)(ncl + 1)))) return rc;
    if ((rc = m->cs_pos.ensure(sizeof(int) * (size_t)cap))) return rc;
    if (split && (rc = m->cs_off_z.ensure(sizeof(int) * (size_t)(nclz + 1)))) return rc;
    p.cs_off = m->cs_off.as<int>();
    p.cs_pos = m->cs_pos.as<int>();
    p.cs_off_z = split ? m->cs_off_z.as<int>() : nullptr;
    HIP_TRY(hipMemsetAsync(m->cs_cnt.as<int>() + ncl, 0, sizeof(int), ctx->stream));
    size_t tb = 0;
    HIP_TRY(launch_scan(nullptr, tb, m->cs_cnt.as<int>(), m->cs_off.as<int>(), (int)(ncl + 1), ctx->stream));
    if ((rc = ctx->temp.ensure(tb))) return rc;
    Params q = p;
    // (a split stream stands across a re-binning that moved nothing only if no shifted-z
    // anchor changed either: RebinBufs::zst[1])
    const bool keep = m->cs_state == 2 && (!split || (m->cs_split && m->zst.p));
    q.items_skip = keep ? m->cs_skip : nullptr;
    q.cs_zflip = m->zst.p ? m->zst.as<int>() + 1 : nullptr;
    q.cs_epoch = m->rb_epoch;
    HIP_TRY(launch_cand_stream(q, (int)ncl, m->cs_cnt.as<int>(), m->cs_off.as<int>(), m->cs_pos.as<int>(), ctx->temp.p,
                               ctx->temp.cap,
                               reinterpret_cast<unsigned long long*>(m->cs_cnt.as<char>() + tot_at), ctx->stream));
    m->cs_state = 1;
    m->cs_split = split;
    return IBTK_LE_OK;
}

static int spread_impl(ibtk_le_ctx ctx, ibtk_le_markers m, int kernel, int centering, int axis,
                       const ibtk_le_patch_geom* geom, double* const* q_dev, int q_depth, const double* Q_dev,
                       int Q_depth, const double* ds_dev, const double* X_dev, bool zero_ghosts, bool zero_first) {
    Params p;
    if (int rc = prepare(ctx, m, kernel, geom, X_dev, p)) return rc;
    p.zero_ghosts = zero_ghosts ? 1 : 0;
    p.zero_first = zero_first ? 1 : 0;
    const int nc = ncomponents(geom, centering, q_depth, Q_depth);
    if (nc < 0) return -nc;
    if (m->n == 0) return IBTK_LE_OK;  // LEInteractor.cpp:2747
    if (!Q_dev || !q_dev) return fail(IBTK_LE_ERR_ARG, "null Q or q");
    if (set_device(ctx)) return IBTK_LE_ERR_DEVICE;
    p.Qin = Q_dev;
    p.ds = ds_dev;
    p.Q_depth = Q_depth;
    p.nsorted = m->n;
    {
        if (int rc = ctx->fbuf.ensure(sizeof(double) * (size_t)m->n * (size_t)std::min(nc, MAXC))) return rc;
        p.sorted_F = ctx->fbuf.as<double>();
    }
    if (geom->ndim == 2) {
        if (int rc = build_candidates(ctx, m, p)) return rc;
        p.cand_off = m->cand_off.as<int>();
        p.cand_idx = m->cand_idx.as<int>();
    }
    ctx->ev_valid = false;
    for (int first = 0; first < nc; first += MAXC) {
        const int cnt = std::min(MAXC, nc - first);
        if (int rc = make_comps(geom, centering, axis, q_dev, q_depth, Q_depth, first, cnt, p)) return rc;
        const bool side = geom->ndim == 3 && side_gather(ctx, m) && !cand_stream_built(m);
        if (side)
            if (int rc = gather_fork(ctx, p)) return rc;
        if (geom->ndim == 3)
            if (int rc = cand_stream(ctx, m, p)) return rc;
        if (side)
            if (int rc = gather_join(ctx)) return rc;
        const bool t = ctx->timing && first == 0;
        const size_t nst = (size_t)m->item_bound * cnt * 8;
        if (geom->ndim == 3)
            if (int rc = stamps_begin(ctx, nst, p)) return rc;
        if (geom->ndim == 3) {
            if (int rc = adds_begin(ctx, p, first == 0)) return rc;
            HIP_TRY(launch_spread_sweep(kernel, p, ctx->stream, t ? ctx->ev0 : nullptr, t ? ctx->ev1 : nullptr,
                                        !side));
            if (int rc = adds_end(ctx, p)) return rc;
        } else {
            HIP_TRY(launch_spread(geom->ndim, kernel, p, ctx->stream, t ? ctx->ev0 : nullptr, t ? ctx->ev1 : nullptr));
        }
        if (int rc = stamps_report(ctx, nst, p)) return rc;
        if (t) ctx->ev_valid = true;
    }
    return IBTK_LE_OK;
}

// ---------------------------------------------------------------------------
// a level of patches: LDataManager::spread / interp's patch loop
// (LDataManager.cpp:625-660, 763-807) as one launch per sweep
// ---------------------------------------------------------------------------
// The device patch table follows the host one; an upload (a pageable copy, which
// waits for the stream) only when the content changed -- a level reused with the
// same arrays uploads nothing per call.
static int upload_patches(ibtk_le_ctx ctx, ibtk_le_markers m) {
    const size_t bytes = sizeof(PatchDesc) * m->pdh.size();
    if (m->pdh_dev.size() == m->pdh.size() && std::memcmp(m->pdh_dev.data(), m->pdh.data(), bytes) == 0)
        return IBTK_LE_OK;
    if (int rc = m->pd.ensure(bytes)) return rc;
    m->pdh_dev = m->pdh;
    HIP_TRY(hipMemcpyAsync(m->pd.p, m->pdh_dev.data(), bytes, hipMemcpyHostToDevice, ctx->stream));
    return IBTK_LE_OK;
}

extern "C" int ibtk_le_level_bin(ibtk_le_ctx ctx, ibtk_le_markers m, int npatch, const ibtk_le_patch_geom* geoms,
                                 int kernel, const double* X_dev, const int* entry_offsets, const int* indices_dev,
                                 const double* Xshift_dev) {
    if (!ctx || !m || !geoms || !entry_offsets) return fail(IBTK_LE_ERR_ARG, "level_bin: null argument");
    if (npatch <= 0) return fail(IBTK_LE_ERR_ARG, "level_bin: no patches");
    if (kernel < 0 || kernel >= K_COUNT) return fail(IBTK_LE_ERR_UNKNOWN_KERNEL, "Unknown kernel function %d", kernel);
    for (int q = 0; q < npatch; ++q) {
        if (int rc = check_geom(&geoms[q])) return rc;
        if (!packed(&geoms[q])) return fail(IBTK_LE_ERR_ARG, "level calls take packed arrays (pitch {0, 0})");
        if (geoms[q].ndim != 3) return fail(IBTK_LE_ERR_ARG, "level_bin: 3-D patches only");
        for (int d = 0; d < 3; ++d)
            if (geoms[q].dx[d] != geoms[0].dx[d]) return fail(IBTK_LE_ERR_ARG, "level_bin: patches of one level share dx");
        if (entry_offsets[q + 1] < entry_offsets[q]) return fail(IBTK_LE_ERR_ARG, "level_bin: decreasing offsets");
    }
    if (entry_offsets[0] != 0) return fail(IBTK_LE_ERR_ARG, "level_bin: entry_offsets[0] must be 0");
    const int n = entry_offsets[npatch];
    if (n > 0 && !X_dev) return fail(IBTK_LE_ERR_ARG, "null X");
    if (set_device(ctx)) return IBTK_LE_ERR_DEVICE;
    const hipStream_t s = ctx->stream;
    m->npatch = npatch;
    m->geoms.assign(geoms, geoms + npatch);
    std::vector<PatchDesc> prev;
    prev.swap(m->pdh);
    m->pdh.assign((size_t)npatch, PatchDesc{});
    long long nb = 0, nj = 0, nz = 0;
    BinGeom bg0{};
    for (int q = 0; q < npatch; ++q) {
        BinGeom bg;
        ColGeom cg;
        if (int rc = make_col_geom(&geoms[q], kernel, bg, cg)) return rc;
        if (q == 0) bg0 = bg;
        PatchDesc& P = m->pdh[q];
        std::memset(&P, 0, sizeof(P));
        P.cg = cg;
        P.bucket_base = (int)nb;
        P.ca_base_z = (int)nz;
        P.jbase = (int)nj;
        sweep_segments(cg, P.S, P.nseg, ctx->tune.seg_items, true);
        for (int d = 0; d < 3; ++d) {
            P.xlo[d] = geoms[q].x_lower[d];
            P.ilower[d] = geoms[q].ilower[d];
        }
        if (prev.size() == (size_t)npatch) std::memcpy(P.comp, prev[q].comp, sizeof(P.comp));  // arrays of the last call
        nb += cg.nbuckets;
        nz += (long long)cg.ncol * (cg.nz + 1);
        nj += (long long)cg.ncol * P.nseg;
        if (nb + 1 >= (1LL << 31) || nj >= (1LL << 30)) return fail(IBTK_LE_ERR_RANGE, "level too large for 31-bit keys");
    }
    m->nbuckets_total = (int)nb;
    m->nclz = nz;
    m->njobs = (int)nj;
    m->n = n;
    m->kernel = kernel;
    m->ndim = 3;
    m->bg = bg0;
    m->cg = m->pdh[0].cg;
    m->S = m->pdh[0].S;
    m->nseg = m->pdh[0].nseg;
    m->geom = geoms[0];
    m->has_indices = indices_dev != nullptr;
    m->has_xshift = Xshift_dev != nullptr;
    m->cand_valid = false;
    m->dedup_done = false;
    m->qin_valid = false;
    m->sel_cached = false;
    m->has_dups = false;
    m->n_dev = nullptr;
    m->binned3 = true;
    int rc;
    if ((rc = upload_patches(ctx, m))) return rc;
    if (m->off_dev.size() != (size_t)(npatch + 1) ||
        std::memcmp(m->off_dev.data(), entry_offsets, sizeof(int) * (size_t)(npatch + 1)) != 0) {
        if ((rc = m->entry_off.ensure(sizeof(int) * (size_t)(npatch + 1)))) return rc;
        m->off_dev.assign(entry_offsets, entry_offsets + npatch + 1);
        HIP_TRY(hipMemcpyAsync(m->entry_off.p, m->off_dev.data(), sizeof(int) * (size_t)(npatch + 1),
                               hipMemcpyHostToDevice, s));
    }
    if ((rc = m->plane_start.ensure(sizeof(int) * (size_t)(nb + 1)))) return rc;
    if (n == 0) {
        HIP_TRY(hipMemsetAsync(m->plane_start.p, 0, sizeof(int) * (size_t)(nb + 1), s));
        return build_items(ctx, m, kernel);
    }
    if ((rc = m->sorted_key.ensure(sizeof(unsigned) * (size_t)n))) return rc;
    if ((rc = m->sorted_l.ensure(sizeof(int) * (size_t)n))) return rc;
    if ((rc = m->sorted_s.ensure(sizeof(int) * (size_t)n))) return rc;
    if ((rc = m->sorted_X.ensure(sizeof(double) * (size_t)n * 3))) return rc;
    if ((rc = ctx->keys_in.ensure(sizeof(unsigned) * (size_t)n))) return rc;
    if ((rc = ctx->vals_in.ensure(sizeof(int) * (size_t)n))) return rc;
    if (m->has_indices) {
        if ((rc = m->indices.ensure(sizeof(int) * (size_t)n))) return rc;
        HIP_TRY(hipMemcpyAsync(m->indices.p, indices_dev, sizeof(int) * (size_t)n, hipMemcpyDeviceToDevice, s));
    }
    if (m->has_xshift) {
        if ((rc = m->xshift.ensure(sizeof(double) * (size_t)n * 3))) return rc;
        HIP_TRY(hipMemcpyAsync(m->xshift.p, Xshift_dev, sizeof(double) * (size_t)n * 3, hipMemcpyDeviceToDevice, s));
    }
    Params p;
    std::memset(&p, 0, sizeof(p));
    p.bg = bg0;
    p.cg = m->cg;
    p.pd = m->pd.as<PatchDesc>();
    p.npatch = npatch;
    p.entry_off = m->entry_off.as<int>();
    p.nbuckets_total = (int)nb;
    p.X = X_dev;
    p.indices = m->has_indices ? m->indices.as<int>() : nullptr;
    p.Xshift = m->has_xshift ? m->xshift.as<double>() : nullptr;
    HIP_TRY(launch_bin_col(kernel, p, n, ctx->keys_in.as<unsigned>(), ctx->vals_in.as<int>(), s));
    int end_bit = 1;
    while ((1ULL << end_bit) <= (unsigned long long)nb) ++end_bit;
    size_t tb = 0;
    HIP_TRY(launch_sort(nullptr, tb, ctx->keys_in.as<unsigned>(), m->sorted_key.as<unsigned>(), ctx->vals_in.as<int>(),
                        m->sorted_l.as<int>(), n, end_bit, s));
    if ((rc = ctx->temp.ensure(tb))) return rc;
    tb = ctx->temp.cap;
    HIP_TRY(launch_sort(ctx->temp.p, tb, ctx->keys_in.as<unsigned>(), m->sorted_key.as<unsigned>(),
                        ctx->vals_in.as<int>(), m->sorted_l.as<int>(), n, end_bit, s));
    p.sorted_l = m->sorted_l.as<int>();
    if ((rc = gather_buckets(ctx, m, kernel, p, n, (int)nb))) return rc;
    return build_items(ctx, m, kernel);
}

// Params of a level call: the patch table with the component arrays of this
// call (q_dev: the arrays of patch 0, then patch 1, ...; per patch NDIM side or
// edge arrays, or one cell / node array), uploaded in stream order.
static int level_params(ibtk_le_ctx ctx, ibtk_le_markers m, int kernel, int centering, int axis,
                        double* const* q_dev, int q_depth, int Q_depth, const double* X, bool interp, Params& p,
                        int& nc) {
    if (!ctx || !m) return fail(IBTK_LE_ERR_ARG, "null ctx/markers");
    if (!m->npatch) return fail(IBTK_LE_ERR_ARG, "markers were not binned for a level (ibtk_le_level_bin)");
    if (kernel != m->kernel) return fail(IBTK_LE_ERR_ARG, "markers were binned for another kernel");
    if (m->n > 0 && !X) return fail(IBTK_LE_ERR_ARG, "null X");
    nc = ncomponents(&m->geoms[0], centering, q_depth, Q_depth);
    if (nc < 0) return -nc;
    if (nc > MAXC) return fail(IBTK_LE_ERR_ARG, "level calls take at most %d components", MAXC);
    if (!q_dev) return fail(IBTK_LE_ERR_ARG, "null q");
    const int per = (centering == IBTK_LE_SIDE || centering == IBTK_LE_EDGE) ? 3 : 1;
    for (int q = 0; q < m->npatch; ++q) {
        const ibtk_le_patch_geom& g = m->geoms[q];
        if (interp) {  // LEInteractor.cpp:2416-2426
            const int gmin = std::min(g.gcw[0], std::min(g.gcw[1], g.gcw[2]));
            if (gmin < ibtk_le_min_ghost_width(kernel))
                return fail(IBTK_LE_ERR_GHOST_WIDTH, "LEInteractor::interpolate(): insufficient ghost cells in patch %d",
                            q);
        }
        Params t;
        std::memset(&t, 0, sizeof(t));
        if (int rc = make_comps(&g, centering, axis, q_dev + (size_t)q * per, q_depth, Q_depth, 0, nc, t)) return rc;
        std::memcpy(m->pdh[q].comp, t.comp, sizeof(t.comp));
        if (q == 0) std::memcpy(p.comp, t.comp, sizeof(t.comp));
    }
    p.tune = ctx->tune;
    if (set_device(ctx)) return IBTK_LE_ERR_DEVICE;
    if (int rc = upload_patches(ctx, m)) return rc;
    p.ncomp = nc;
    p.bg = m->bg;
    p.cg = m->cg;
    p.S = m->S;
    p.nseg = m->nseg;
    p.pd = m->pd.as<PatchDesc>();
    p.npatch = m->npatch;
    p.entry_off = m->entry_off.as<int>();
    p.nbuckets_total = m->nbuckets_total;
    p.njobs = m->njobs;
    p.items = m->items.as<SweepItem>();
    p.nitems = m->nitems.as<int>();
    p.item_bound = m->item_bound;
    p.nsorted = m->n;
    p.X = X;
    p.indices = m->has_indices ? m->indices.as<int>() : nullptr;
    p.Xshift = m->has_xshift ? m->xshift.as<double>() : nullptr;
    p.sorted_l = m->sorted_l.as<int>();
    p.sorted_s = m->sorted_s.as<int>();
    p.sorted_X = m->sorted_X.as<double>();
    p.sorted_X_ref = m->xcur_set ? m->xcur.as<double*>() : nullptr;
    p.sorted_key = m->sorted_key.as<unsigned>();
    p.plane_start = m->plane_start.as<int>();
    p.err = ctx->err.as<int>();
    p.sink = ctx->sink.as<double>();
    p.K6 = ib6_K();
    p.h3 = (m->geoms[0].dx[0] * m->geoms[0].dx[1]) * m->geoms[0].dx[2];
    p.Q_depth = Q_depth;
    return IBTK_LE_OK;
}

extern "C" int ibtk_le_level_interp(ibtk_le_ctx ctx, ibtk_le_markers m, int kernel, int centering, int axis,
                                    const double* const* q_dev, int q_depth, double* Q_dev, int Q_depth,
                                    const double* X_dev) {
    Params p;
    std::memset(&p, 0, sizeof(p));
    int nc = 0;
    if (int rc = level_params(ctx, m, kernel, centering, axis, const_cast<double* const*>(q_dev), q_depth, Q_depth,
                              X_dev, true, p, nc))
        return rc;
    if (m->n == 0) return IBTK_LE_OK;
    if (!Q_dev) return fail(IBTK_LE_ERR_ARG, "null Q");
    if (m->qin_valid) {  // the interior entries only (each names its marker once)
        p.qdst = m->qin.as<int>();
    } else {
        if (int rc = build_dedup(ctx, m)) return rc;
        p.qdst = m->has_dups ? m->qdst.as<int>() : nullptr;
    }
    p.Qout = Q_dev;
    const bool t = ctx->timing;
    ctx->ev_valid = false;
    HIP_TRY(launch_interp_sweep(kernel, p, m->n, ctx->stream, t ? ctx->ev0 : nullptr, t ? ctx->ev1 : nullptr));
    if (t) ctx->ev_valid = true;
    return IBTK_LE_OK;
}

// LDataManager::interp's patch loop takes each patch's interior list
// (LDataManager.cpp:763-807 with LIndexSetData's interior indices), the spread its
// ghost-box list; the interior list is a sub-list of the ghost-box one (the markers
// whose cell is in the patch box, unshifted).  Rather than binning both, a level
// binned on the ghost-box lists is told which of its entries the interior lists name:
// later level interps write Q from those entries only, and the next bin clears it.
// An interior entry with no match in its patch's binned list raises device flag 4
// (reported by ibtk_le_ctx_synchronize; no host sync here).
// Forget the last selection: the next ibtk_le_level_select_interior recomputes it even if its
// offsets, index pointer and n_markers are the same (the caller rewrote the lists in place, or
// a new list was allocated at the old address)
extern "C" int ibtk_le_level_select_interior_reset(ibtk_le_markers m) {
    if (!m) return fail(IBTK_LE_ERR_ARG, "select_interior_reset: null markers");
    m->sel_cached = false;
    return IBTK_LE_OK;
}

extern "C" int ibtk_le_level_select_interior(ibtk_le_ctx ctx, ibtk_le_markers m, int n_markers,
                                             const int* interior_offsets, const int* interior_indices_dev) {
    if (!ctx || !m || !interior_offsets) return fail(IBTK_LE_ERR_ARG, "select_interior: null argument");
    if (m->npatch <= 0) return fail(IBTK_LE_ERR_ARG, "select_interior: not a level binning (ibtk_le_level_bin)");
    const int np = m->npatch;
    if (interior_offsets[0] != 0) return fail(IBTK_LE_ERR_ARG, "select_interior: offsets[0] must be 0");
    for (int q = 0; q < np; ++q)
        if (interior_offsets[q + 1] < interior_offsets[q]) return fail(IBTK_LE_ERR_ARG, "select_interior: decreasing offsets");
    const int n_int = interior_offsets[np];
    if (n_int > 0 && (!interior_indices_dev || n_markers <= 0))
        return fail(IBTK_LE_ERR_ARG, "select_interior: null indices or no markers");
    if (!m->has_indices) return fail(IBTK_LE_ERR_ARG, "select_interior: the binned lists must be index lists");
    if (set_device(ctx)) return IBTK_LE_ERR_DEVICE;
    const hipStream_t s = ctx->stream;
    int rc;
    if ((rc = m->qin.ensure(sizeof(int) * (size_t)std::max(m->n, 1)))) return rc;
    if ((rc = m->owner.ensure(sizeof(int) * (size_t)std::max(n_markers, 1)))) return rc;
    // the same lists as the last selection since the last full binning: the kernels below
    // return at once on the device unless a re-binning moved something (sel_gs)
    const bool same = m->sel_cached && m->sel_idx == interior_indices_dev && m->sel_nm == n_markers &&
                      m->sel_off.size() == (size_t)(np + 1) &&
                      std::equal(m->sel_off.begin(), m->sel_off.end(), interior_offsets);
    if (!m->sel_gs.p) {
        if ((rc = m->sel_gs.ensure(2 * sizeof(int)))) return rc;
        HIP_TRY(hipMemsetAsync(m->sel_gs.p, 0, sizeof(int), s));
    }
    if (!same) HIP_TRY(hipMemsetAsync(m->sel_gs.as<int>() + 1, 0xff, sizeof(int), s));  // -1: no selection
    const int* gs = m->sel_gs.as<int>();
    if ((rc = m->int_off.ensure(sizeof(int) * (size_t)(np + 1)))) return rc;
    const int nblk = CHECK_STRIPES;  // the kept entries' count, striped over CHECK_STRIPES counters
    if ((rc = ctx->counts.ensure(sizeof(int) * (size_t)nblk))) return rc;
    HIP_TRY(hipMemsetAsync(ctx->counts.p, 0, sizeof(int) * (size_t)nblk, s));
    // owner[] follows the lists alone: with the same lists (a re-binning between regrids moved
    // markers, not the lists) the last selection's stands -- only the targets are redone
    if (!same) {
        HIP_TRY(hipMemcpyAsync(m->int_off.p, interior_offsets, sizeof(int) * (size_t)(np + 1), hipMemcpyHostToDevice,
                               s));
        HIP_TRY(hipMemsetAsync(m->owner.p, 0xff, sizeof(int) * (size_t)std::max(n_markers, 1), s));
        HIP_TRY(launch_interior_owner(m->int_off.as<int>(), np, interior_indices_dev, n_int, n_markers,
                                      m->owner.as<int>(), ctx->err.as<int>(), gs, s));
    }
    // An entry of patch q's list whose marker q owns is a periodic image only if the image
    // (a whole period away) lies in q's ghost box as well: impossible when the level spans
    // more than any patch's ghost box in every dim (a period is at least the level's extent),
    // and then the Xshift rows (a 24-byte gather per entry) need not be read
    bool need_shift = m->has_xshift;
    if (need_shift) {
        bool wide = true;
        for (int d = 0; d < 3 && wide; ++d) {
            int lo = INT_MAX, hi = INT_MIN, gb = 0;
            for (const ibtk_le_patch_geom& g : m->geoms) {
                lo = std::min(lo, g.ilower[d]);
                hi = std::max(hi, g.iupper[d]);
                gb = std::max(gb, g.iupper[d] - g.ilower[d] + 2 + 2 * g.gcw[d]);  // ghost box (+ a face)
            }
            wide = hi - lo + 1 > gb;
        }
        need_shift = !wide;
    }
    HIP_TRY(launch_interior_targets(m->sorted_l.as<int>(), m->sorted_s.as<int>(), m->entry_off.as<int>(), np,
                                    need_shift ? m->xshift.as<double>() : nullptr, m->owner.as<int>(), n_markers,
                                    m->n, m->qin.as<int>(), ctx->counts.as<int>(), ctx->err.as<int>(), gs, s));
    HIP_TRY(launch_check_count(ctx->counts.as<int>(), m->n > 0 ? nblk : 0, n_int, ctx->err.as<int>(), 4, s, gs));
    HIP_TRY(launch_sel_mark(m->sel_gs.as<int>(), s));
    m->qin_valid = true;
    m->sel_cached = true;
    m->sel_idx = interior_indices_dev;
    m->sel_nm = n_markers;
    m->sel_off.assign(interior_offsets, interior_offsets + np + 1);
    return IBTK_LE_OK;
}

static int level_spread_impl(ibtk_le_ctx ctx, ibtk_le_markers m, int kernel, int centering, int axis,
                             double* const* q_dev, int q_depth, const double* Q_dev, int Q_depth, const double* X_dev,
                             bool zero_first) {
    Params p;
    std::memset(&p, 0, sizeof(p));
    int nc = 0;
    if (int rc = level_params(ctx, m, kernel, centering, axis, q_dev, q_depth, Q_depth, X_dev, false, p, nc))
        return rc;
    if (m->n == 0)  // nothing to spread: LEInteractor.cpp:2747 (zero_first: the zeroing alone)
        return zero_first ? ibtk_le_level_zero(ctx, m->npatch, m->geoms.data(), centering, q_dev, q_depth) : IBTK_LE_OK;
    if (!Q_dev) return fail(IBTK_LE_ERR_ARG, "null Q");
    p.Qin = Q_dev;
    p.zero_first = zero_first ? 1 : 0;
    {
        if (int rc = ctx->fbuf.ensure(sizeof(double) * (size_t)m->n * (size_t)nc)) return rc;
        p.sorted_F = ctx->fbuf.as<double>();
    }
    const bool side = side_gather(ctx, m) && !cand_stream_built(m);
    if (side)
        if (int rc = gather_fork(ctx, p)) return rc;
    if (int rc = cand_stream(ctx, m, p)) return rc;
    if (side)
        if (int rc = gather_join(ctx)) return rc;
    const bool t = ctx->timing;
    ctx->ev_valid = false;
    const size_t nst = (size_t)m->item_bound * nc * 8;
    if (int rc = stamps_begin(ctx, nst, p)) return rc;
    if (int rc = adds_begin(ctx, p, true)) return rc;
    HIP_TRY(launch_spread_sweep(kernel, p, ctx->stream, t ? ctx->ev0 : nullptr, t ? ctx->ev1 : nullptr, !side));
    if (int rc = adds_end(ctx, p)) return rc;
    if (int rc = stamps_report(ctx, nst, p)) return rc;
    if (t) ctx->ev_valid = true;
    return IBTK_LE_OK;
}

extern "C" int ibtk_le_level_spread(ibtk_le_ctx ctx, ibtk_le_markers m, int kernel, int centering, int axis,
                                    double* const* q_dev, int q_depth, const double* Q_dev, int Q_depth,
                                    const double* X_dev) {
    return level_spread_impl(ctx, m, kernel, centering, axis, q_dev, q_depth, Q_dev, Q_depth, X_dev, false);
}

// LDataManager::spread's setToScalar(f, 0, interior_only = false) and its patch loop
// of LEInteractor::spread (LDataManager.cpp:588-654) fused: the sweep's items start
// their owned points from 0 instead of reading them, and the items no marker reaches
// store zeros.  Bitwise ibtk_le_level_zero followed by ibtk_le_level_spread.
extern "C" int ibtk_le_level_zero_spread(ibtk_le_ctx ctx, ibtk_le_markers m, int kernel, int centering, int axis,
                                         double* const* q_dev, int q_depth, const double* Q_dev, int Q_depth,
                                         const double* X_dev) {
    return level_spread_impl(ctx, m, kernel, centering, axis, q_dev, q_depth, Q_dev, Q_depth, X_dev, true);
}

// Ghost fill of a level of equal patches tiling a box (periodic in the flagged
// dims): LDataManager::interp's fill schedule (LDataManager.cpp:748-751).
// q_dev as for ibtk_le_level_interp.  The device tables live in the context
// until the next call with another tiling.
// The tiling of a level of equal patches tiling a box (periodic in the flagged dims):
// cells per patch, tiles per dim, tile of each patch and patch of each tile (-1: none).
static int level_tiling(int npatch, const ibtk_le_patch_geom* geoms, int centering, const int* periodic,
                        const char* who, LevelTiling& t, std::vector<int>& tile_of, std::vector<int>& patch_of) {
    std::memset(&t, 0, sizeof(t));
    int lo[3] = {INT_MAX, INT_MAX, INT_MAX}, hi[3] = {INT_MIN, INT_MIN, INT_MIN};
    for (int q = 0; q < npatch; ++q) {
        if (int rc = check_geom(&geoms[q])) return rc;
        if (!packed(&geoms[q])) return fail(IBTK_LE_ERR_ARG, "level calls take packed arrays (pitch {0, 0})");
        if (geoms[q].ndim != 3) return fail(IBTK_LE_ERR_ARG, "%s: 3-D patches", who);
        for (int d = 0; d < 3; ++d) {
            const int n = geoms[q].iupper[d] - geoms[q].ilower[d] + 1;
            if (q == 0) t.n[d] = n;
            if (n != t.n[d] || geoms[q].gcw[d] != geoms[0].gcw[0])
                return fail(IBTK_LE_ERR_ARG, "%s: equal patches and ghost widths only", who);
            lo[d] = std::min(lo[d], geoms[q].ilower[d]);
            hi[d] = std::max(hi[d], geoms[q].iupper[d]);
        }
    }
    t.g = geoms[0].gcw[0];
    long long ntiles = 1;
    for (int d = 0; d < 3; ++d) {
        t.dom_lo[d] = lo[d];
        t.ntile[d] = (hi[d] - lo[d] + 1) / t.n[d];
        if (t.ntile[d] * t.n[d] != hi[d] - lo[d] + 1 || t.g > t.n[d])
            return fail(IBTK_LE_ERR_ARG, "%s: the patches must tile a box, ghost width <= patch size", who);
        t.periodic[d] = periodic ? periodic[d] != 0 : 1;
        ntiles *= t.ntile[d];
    }
    tile_of.assign(npatch, 0);
    patch_of.assign((size_t)ntiles, -1);
    for (int q = 0; q < npatch; ++q) {
        int tc[3];
        for (int d = 0; d < 3; ++d) {
            tc[d] = (geoms[q].ilower[d] - lo[d]) / t.n[d];
            if ((geoms[q].ilower[d] - lo[d]) % t.n[d]) return fail(IBTK_LE_ERR_ARG, "%s: unaligned patch", who);
        }
        tile_of[q] = tc[0] + t.ntile[0] * (tc[1] + t.ntile[1] * tc[2]);
        if (patch_of[tile_of[q]] >= 0) return fail(IBTK_LE_ERR_ARG, "%s: overlapping patches", who);
        patch_of[tile_of[q]] = q;
    }
    t.side = centering == IBTK_LE_SIDE;
    t.ncomp = t.side ? 3 : 1;
    return IBTK_LE_OK;
}

// the patch supplying patch q's ghost points in direction dir (per dim -1, 0, +1), as
// k_level_fill finds it: wrapped in the periodic dims, none (-1) across another face
static int level_neighbour(const LevelTiling& t, const std::vector<int>& tile_of, const std::vector<int>& patch_of,
                           int q, const int dir[3]) {
    const int tile = tile_of[q];
    const int tc[3] = {tile % t.ntile[0], (tile / t.ntile[0]) % t.ntile[1], tile / (t.ntile[0] * t.ntile[1])};
    int nt[3];
    for (int d = 0; d < 3; ++d) {
        nt[d] = tc[d] + dir[d];
        if (nt[d] < 0 || nt[d] >= t.ntile[d]) {
            if (!t.periodic[d]) return -1;
            nt[d] = (nt[d] + t.ntile[d]) % t.ntile[d];
        }
    }
    return patch_of[nt[0] + t.ntile[0] * (nt[1] + t.ntile[1] * nt[2])];
}

// Ghost fill of a level of equal patches tiling a box (periodic in the flagged
// dims): LDataManager::interp's fill schedule (LDataManager.cpp:748-751).
// q_dev as for ibtk_le_level_interp.  The device tables live in the context
// until the next call with another tiling.
extern "C" int ibtk_le_level_fill_ghosts(ibtk_le_ctx ctx, int npatch, const ibtk_le_patch_geom* geoms,
                                         int centering, double* const* q_dev, int q_depth, const int* periodic) {
    if (!ctx || !geoms || !q_dev || npatch <= 0) return fail(IBTK_LE_ERR_ARG, "level_fill_ghosts: null argument");
    if (centering != IBTK_LE_SIDE && centering != IBTK_LE_CELL)
        return fail(IBTK_LE_ERR_ARG, "level_fill_ghosts: side or cell data");
    LevelTiling t;
    std::vector<int> tile_of, patch_of;
    if (int rc = level_tiling(npatch, geoms, centering, periodic, "level_fill_ghosts", t, tile_of, patch_of)) return rc;
    const long long ntiles = (long long)patch_of.size();
    const size_t narr = (size_t)npatch * t.ncomp;
    for (size_t i = 0; i < narr; ++i)
        if (!q_dev[i]) return fail(IBTK_LE_ERR_ARG, "level_fill_ghosts: null array");
    if (set_device(ctx)) return IBTK_LE_ERR_DEVICE;
    const hipStream_t s = ctx->stream;
    int rc;
    if ((rc = ctx->lvl_tab.ensure(sizeof(int) * (size_t)(npatch + ntiles) + sizeof(double*) * narr + 64))) return rc;
    char* base = ctx->lvl_tab.as<char>();
    double** arr_d = reinterpret_cast<double**>(base);
    int* tile_d = reinterpret_cast<int*>(base + sizeof(double*) * narr);
    int* patch_d = tile_d + npatch;
    // upload the tables only when they changed (a pageable copy waits for the stream)
    std::vector<char> host(sizeof(double*) * narr + sizeof(int) * (size_t)(npatch + ntiles));
    std::memcpy(host.data(), q_dev, sizeof(double*) * narr);
    std::memcpy(host.data() + sizeof(double*) * narr, tile_of.data(), sizeof(int) * (size_t)npatch);
    std::memcpy(host.data() + sizeof(double*) * narr + sizeof(int) * (size_t)npatch, patch_of.data(),
                sizeof(int) * (size_t)ntiles);
    if (ctx->lvl_host != host) {
        ctx->lvl_host = host;
        HIP_TRY(hipMemcpyAsync(base, ctx->lvl_host.data(), host.size(), hipMemcpyHostToDevice, s));
    }
    HIP_TRY(launch_level_fill(t, npatch, tile_d, patch_d, arr_d, t.side ? 1 : q_depth, s));
    return IBTK_LE_OK;
}

// ibtk_le_level_fill_ghosts followed by ibtk_le_level_interp, Q bit for bit, in one
// sweep: a ghost point of a patch is read in the neighbour patch that the fill would
// copy it from (k_level_fill's rule: the patch owning its wrapped cell, at the same
// global index), so no ghost layer is written or read twice.  Needs, per component,
// every patch's array within one 2-GB window (e.g. one allocation per component for the
// level) and patches of at least (32 + W - 1) x (COLY + W - 1) cells in x and y;
// otherwise, or for cell data of depth > 1, the two calls.
extern "C" int ibtk_le_level_fill_interp(ibtk_le_ctx ctx, ibtk_le_markers m, int kernel, int centering, int axis,
                                         double* const* q_dev, int q_depth, double* Q_dev, int Q_depth,
                                         const double* X_dev, const int* periodic) {
    if (!ctx || !m || !q_dev) return fail(IBTK_LE_ERR_ARG, "level_fill_interp: null argument");
    if (m->npatch <= 0) return fail(IBTK_LE_ERR_ARG, "level_fill_interp: not a level binning (ibtk_le_level_bin)");
    const int np = m->npatch;
    auto unfused = [&]() {
        if (int rc = ibtk_le_level_fill_ghosts(ctx, np, m->geoms.data(), centering, q_dev, q_depth, periodic)) return rc;
        return ibtk_le_level_interp(ctx, m, kernel, centering, axis, q_dev, q_depth, Q_dev, Q_depth, X_dev);
    };
    if ((centering != IBTK_LE_SIDE && centering != IBTK_LE_CELL) || (centering == IBTK_LE_CELL && q_depth != 1))
        return unfused();
    LevelTiling t;
    std::vector<int> tile_of, patch_of;
    if (int rc = level_tiling(np, m->geoms.data(), centering, periodic, "level_fill_interp", t, tile_of, patch_of))
        return rc;
    {  // a staged column region (COLX + HI - LO by COLY + HI - LO points) crosses at most one
       // face of its patch per dim (le_sweep.hip, the interp's level-fill staging)
        const KernelInfo ki = kKernelInfo[kernel < 0 || kernel >= K_COUNT ? 0 : kernel];
        if (t.n[0] < COLX + ki.HI - ki.LO || t.n[1] < COLY + ki.HI - ki.LO) return unfused();
    }
    Params p;
    std::memset(&p, 0, sizeof(p));
    int nc = 0;
    if (int rc = level_params(ctx, m, kernel, centering, axis, q_dev, q_depth, Q_depth, X_dev, true, p, nc)) return rc;
    if (m->n == 0) return IBTK_LE_OK;
    if (!Q_dev) return fail(IBTK_LE_ERR_ARG, "null Q");
    // each component's window: its arrays' lowest start to highest end, below 2 GB
    // (buffer offsets are 32-bit and OFF_NONE is 2^31)
    const int per = t.side ? 3 : 1;
    uintptr_t wlo[MAXC], whi[MAXC];
    for (int c = 0; c < nc; ++c) {
        wlo[c] = UINTPTR_MAX;
        whi[c] = 0;
        for (int q = 0; q < np; ++q) {
            const CompDesc& cd = m->pdh[q].comp[c];
            const uintptr_t a = reinterpret_cast<uintptr_t>(cd.u);
            const uintptr_t b = a + sizeof(double) * (size_t)cd.s2 * (size_t)(cd.hi[2] - cd.lo[2] + 1);
            wlo[c] = std::min(wlo[c], a);
            whi[c] = std::max(whi[c], b);
        }
        if (whi[c] - wlo[c] >= (uintptr_t(1) << 31)) return unfused();
    }
    (void)per;
    // the record per component and patch (le_sweep.hip LVL_REC): the 27 suppliers, the window
    constexpr int REC = 32;
    std::vector<int2> tab((size_t)nc * np * REC, make_int2(0, 0));
    for (int c = 0; c < nc; ++c)
        for (int q = 0; q < np; ++q) {
            int2* r = tab.data() + ((size_t)c * np + q) * REC;
            for (int k = 0; k < 27; ++k) {
                const int dir[3] = {k % 3 - 1, (k / 3) % 3 - 1, k / 9 - 1};
                const int sq = k == 13 ? -1 : level_neighbour(t, tile_of, patch_of, q, dir);
                const CompDesc& src = m->pdh[sq >= 0 ? sq : q].comp[c];
                r[k] = make_int2((int)(reinterpret_cast<uintptr_t>(src.u) - wlo[c]), sq >= 0 ? 1 : 0);
            }
            const uint64_t b = (uint64_t)wlo[c];
            r[27] = make_int2((int)(unsigned)(b & 0xffffffffu), (int)(unsigned)(b >> 32));
            r[28] = make_int2((int)(unsigned)(whi[c] - wlo[c]), 0);
        }
    if (set_device(ctx)) return IBTK_LE_ERR_DEVICE;
    const size_t bytes = sizeof(int2) * tab.size();
    if (int rc = m->lvl_nbr.ensure(bytes)) return rc;
    if (m->lvl_nbr_host.size() != tab.size() || std::memcmp(m->lvl_nbr_host.data(), tab.data(), bytes) != 0) {
        m->lvl_nbr_host = tab;  // a pageable copy waits for the stream: only when changed
        HIP_TRY(hipMemcpyAsync(m->lvl_nbr.p, m->lvl_nbr_host.data(), bytes, hipMemcpyHostToDevice, ctx->stream));
    }
    p.lvl_nbr = m->lvl_nbr.as<int2>();
    for (int d = 0; d < 3; ++d) p.lvl_n[d] = t.n[d];
    if (m->qin_valid) {
        p.qdst = m->qin.as<int>();
    } else {
        if (int rc = build_dedup(ctx, m)) return rc;
        p.qdst = m->has_dups ? m->qdst.as<int>() : nullptr;
    }
    p.Qout = Q_dev;
    const bool tm = ctx->timing;
    ctx->ev_valid = false;
    HIP_TRY(launch_interp_sweep(kernel, p, m->n, ctx->stream, tm ? ctx->ev0 : nullptr, tm ? ctx->ev1 : nullptr));
    if (tm) ctx->ev_valid = true;
    return IBTK_LE_OK;
}

extern "C" int ibtk_le_level_zero(ibtk_le_ctx ctx, int npatch, const ibtk_le_patch_geom* geoms, int centering,
                                  double* const* q_dev, int q_depth) {
    if (!ctx || !geoms || !q_dev || npatch <= 0) return fail(IBTK_LE_ERR_ARG, "level_zero: null argument");
    if (q_depth < 1) return fail(IBTK_LE_ERR_ARG, "level_zero: q_depth < 1");
    const int nd = geoms[0].ndim;
    const bool vec = centering == IBTK_LE_SIDE || centering == IBTK_LE_EDGE;
    if (!vec && centering != IBTK_LE_CELL && centering != IBTK_LE_NODE)
        return fail(IBTK_LE_ERR_ARG, "level_zero: unknown centering %d", centering);
    const int per = vec ? nd : 1;
    const size_t narr = (size_t)npatch * per;
    if (narr > 65535) return fail(IBTK_LE_ERR_RANGE, "level_zero: more than 65535 arrays");
    std::vector<long long> cnt(narr);
    long long mx = 0;
    for (int q = 0; q < npatch; ++q) {
        if (int rc = check_geom(&geoms[q])) return rc;
        if (!packed(&geoms[q])) return fail(IBTK_LE_ERR_ARG, "level calls take packed arrays (pitch {0, 0})");
        if (geoms[q].ndim != nd) return fail(IBTK_LE_ERR_ARG, "level_zero: patches of one dimension");
        for (int a = 0; a < per; ++a) {
            long long n = vec ? 1 : q_depth;
            for (int d = 0; d < nd; ++d) {
                const int cells = geoms[q].iupper[d] - geoms[q].ilower[d] + 1;
                int extra = 0;  // the extra point along the centring's dims
                if (centering == IBTK_LE_NODE) extra = 1;
                else if (centering == IBTK_LE_SIDE) extra = d == a;
                else if (centering == IBTK_LE_EDGE) extra = d != a;
                n *= cells + extra + 2 * geoms[q].gcw[d];
            }
            if (!q_dev[(size_t)q * per + a]) return fail(IBTK_LE_ERR_ARG, "level_zero: null array");
            cnt[(size_t)q * per + a] = n;
            mx = std::max(mx, n);
        }
    }
    if (set_device(ctx)) return IBTK_LE_ERR_DEVICE;
    const size_t bytes = sizeof(double*) * narr + sizeof(long long) * narr;
    int rc;
    if ((rc = ctx->zero_tab.ensure(bytes))) return rc;
    std::vector<char> host(bytes);
    std::memcpy(host.data(), q_dev, sizeof(double*) * narr);
    std::memcpy(host.data() + sizeof(double*) * narr, cnt.data(), sizeof(long long) * narr);
    if (ctx->zero_host != host) {  // a pageable copy waits for the stream: only when changed
        ctx->zero_host = host;
        HIP_TRY(hipMemcpyAsync(ctx->zero_tab.p, ctx->zero_host.data(), bytes, hipMemcpyHostToDevice, ctx->stream));
    }
    char* base = ctx->zero_tab.as<char>();
    HIP_TRY(launch_level_zero(reinterpret_cast<double* const*>(base),
                              reinterpret_cast<const long long*>(base + sizeof(double*) * narr), (int)narr, mx,
                              ctx->stream));
    return IBTK_LE_OK;
}

// ---------------------------------------------------------------------------
// periodic helpers
// ---------------------------------------------------------------------------
static int ghost_descs(const ibtk_le_patch_geom* g, int centering, double* const* q, int q_depth, GhostDesc* out,
                       int* nout) {
    const int nd = g->ndim;
    int narr = 0;
    for (int a = 0;; ++a) {
        int ext_mask = 0;
        double* base = nullptr;
        int depth = 1;
        if (centering == IBTK_LE_CELL || centering == IBTK_LE_NODE) {
            if (a > 0) break;
            base = q[0];
            depth = q_depth;
            ext_mask = centering == IBTK_LE_NODE ? (1 << nd) - 1 : 0;
        } else if (centering == IBTK_LE_SIDE || centering == IBTK_LE_EDGE) {
            if (a >= nd) break;
            base = q[a];
            ext_mask = centering == IBTK_LE_SIDE ? (1 << a) : (((1 << nd) - 1) & ~(1 << a));
        } else {
            return fail(IBTK_LE_ERR_ARG, "unknown centering %d", centering);
        }
        if (!base) return fail(IBTK_LE_ERR_ARG, "null Eulerian array");
        int64_t n[3] = {1, 1, 1};
        GhostDesc gd;
        std::memset(&gd, 0, sizeof(gd));
        for (int d = 0; d < nd; ++d) {
            gd.lo[d] = g->ilower[d] - g->gcw[d];
            gd.hi[d] = g->iupper[d] + g->gcw[d] + ((ext_mask >> d) & 1);
            gd.ilo[d] = g->ilower[d];
            gd.ihi[d] = g->iupper[d];
            n[d] = gd.hi[d] - gd.lo[d] + 1;
        }
        int64_t sd;
        array_strides(g, n, gd.s1, gd.s2, sd);
        for (int k = 0; k < depth; ++k) {
            if (narr >= 16) return fail(IBTK_LE_ERR_ARG, "too many arrays");
            out[narr] = gd;
            out[narr].u = base + (int64_t)k * sd;
            ++narr;
        }
    }
    *nout = narr;
    return IBTK_LE_OK;
}

static int ghost_op(ibtk_le_ctx ctx, const ibtk_le_patch_geom* geom, int centering, double* const* q, int q_depth,
                    const int* periodic, int mode) {
    if (!ctx || !q) return fail(IBTK_LE_ERR_ARG, "null argument");
    if (int rc = check_geom(geom)) return rc;
    if (set_device(ctx)) return IBTK_LE_ERR_DEVICE;
    GhostDesc gds[16];
    int n = 0;
    if (int rc = ghost_descs(geom, centering, q, q_depth, gds, &n)) return rc;
    int per[3] = {1, 1, 1};
    if (periodic)
        for (int d = 0; d < geom->ndim; ++d) per[d] = periodic[d];
    for (int d = 0; d < geom->ndim; ++d)
        if (per[d] && geom->iupper[d] - geom->ilower[d] + 1 < 2 * geom->gcw[d] + 1)
            return fail(IBTK_LE_ERR_ARG, "periodic dim %d narrower than 2*ghost+1", d);
    if (mode == 0) HIP_TRY(launch_fill_periodic(geom->ndim, gds, n, per, ctx->stream));
    else if (mode == 1) HIP_TRY(launch_fold_periodic(geom->ndim, gds, n, per, ctx->stream));
    else HIP_TRY(launch_zero_ghosts(geom->ndim, gds, n, ctx->stream));
    return IBTK_LE_OK;
}

extern "C" int ibtk_le_fill_periodic_ghosts(ibtk_le_ctx ctx, const ibtk_le_patch_geom* geom, int centering,
                                            double* const* q_dev, int q_depth, const int* periodic) {
    return ghost_op(ctx, geom, centering, q_dev, q_depth, periodic, 0);
}
extern "C" int ibtk_le_fold_periodic_ghosts(ibtk_le_ctx ctx, const ibtk_le_patch_geom* geom, int centering,
                                            double* const* q_dev, int q_depth, const int* periodic) {
    return ghost_op(ctx, geom, centering, q_dev, q_depth, periodic, 1);
}
// CartSideRobinPhysBdryOp::setPhysicalBoundaryConditions (adjoint = 0,
// CartSideRobinPhysBdryOp.cpp:358-422) and accumulateFromPhysicalBoundaryData
// (adjoint = 1, :429-493) on one patch of side data.
extern "C" int ibtk_le_phys_bdry_side(ibtk_le_ctx ctx, const ibtk_le_patch_geom* geom, double* const* u_dev,
                                      const int* physical, const double* acoef, const double* bcoef,
                                      const double* gcoef, int adjoint) {
    if (!ctx || !u_dev || !physical || !acoef || !bcoef || !gcoef) return fail(IBTK_LE_ERR_ARG, "null argument");
    if (int rc = check_geom(geom)) return rc;
    const int nd = geom->ndim, g = geom->gcw[0];
    for (int d = 1; d < nd; ++d)  // CartSideRobinPhysBdryOp.cpp:519-527
        if (geom->gcw[d] != g) return fail(IBTK_LE_ERR_GHOST_WIDTH, "non-uniform ghost cell widths");
    if (g > 16) return fail(IBTK_LE_ERR_GHOST_WIDTH, "ghost width %d above 16", g);
    if (g == 0) return IBTK_LE_OK;  // ghost_width_to_fill == 0 (:432)
    BdSide P;
    std::memset(&P, 0, sizeof(P));
    P.ndim = nd;
    P.g = g;
    for (int d = 0; d < nd; ++d) {
        P.ilo[d] = geom->ilower[d];
        P.ihi[d] = geom->iupper[d];
        P.dx[d] = geom->dx[d];
    }
    for (int c = 0; c < nd; ++c) {
        if (!u_dev[c]) return fail(IBTK_LE_ERR_ARG, "null side array %d", c);
        P.u[c] = u_dev[c];
        int64_t n[3] = {1, 1, 1};
        for (int d = 0; d < nd; ++d) {
            P.lo[c][d] = P.ilo[d] - g;
            n[d] = (int64_t)(P.ihi[d] - P.ilo[d] + 1 + 2 * g + (d == c ? 1 : 0));
        }
        int64_t sd;
        array_strides(geom, n, P.s1[c], P.s2[c], sd);
    }
    int phys[6] = {0, 0, 0, 0, 0, 0};
    BdCoef coef[18];
    for (int loc = 0; loc < 2 * nd; ++loc) phys[loc] = physical[loc] != 0;
    for (int i = 0; i < nd * 2 * nd; ++i) coef[i] = BdCoef{acoef[i], bcoef[i], gcoef[i]};
    if (set_device(ctx)) return IBTK_LE_ERR_DEVICE;
    HIP_TRY(launch_phys_bdry_side(P, phys, coef, adjoint ? 1 : 0, ctx->stream));
    return IBTK_LE_OK;
}
extern "C" int ibtk_le_position_update(ibtk_le_ctx ctx, int scheme, long long n, double dt, const double* X_cur_dev,
                                       const double* U0_dev, const double* U1_dev, double* X_new_dev) {
    if (!ctx) return fail(IBTK_LE_ERR_ARG, "null context");
    if (scheme < IBTK_LE_EULER || scheme > IBTK_LE_TRAPEZOIDAL) return fail(IBTK_LE_ERR_ARG, "unknown update scheme");
    if (n < 0) return fail(IBTK_LE_ERR_ARG, "negative length");
    if (n == 0) return IBTK_LE_OK;
    if (!X_cur_dev || !U0_dev || !X_new_dev || (scheme == IBTK_LE_TRAPEZOIDAL && !U1_dev))
        return fail(IBTK_LE_ERR_ARG, "null array");
    HIP_TRY(hipSetDevice(ctx->device));
    HIP_TRY(launch_position_update(scheme, (long)n, dt, X_cur_dev, U0_dev, U1_dev, X_new_dev, ctx->stream));
    return IBTK_LE_OK;
}

static int slab_update_partition_impl(ibtk_le_ctx ctx, int scheme, long long M, double dt, const double* X_cur_dev,
                                      const double* U0_dev, const double* U1_dev, double* X_new_dev, const double* L,
                                      int Nz, int nranks, int rank, const int* n_dev, int* order_dev, int* counts_dev);

extern "C" int ibtk_le_slab_update_partition(ibtk_le_ctx ctx, int scheme, long long M, double dt,
                                             const double* X_cur_dev, const double* U0_dev, const double* U1_dev,
                                             double* X_new_dev, const double* L, int Nz, int nranks, int rank,
                                             int* order_dev, int* counts_dev) {
    return slab_update_partition_impl(ctx, scheme, M, dt, X_cur_dev, U0_dev, U1_dev, X_new_dev, L, Nz, nranks, rank,
                                      nullptr, order_dev, counts_dev);
}

extern "C" int ibtk_le_slab_update_partition_count(ibtk_le_ctx ctx, int scheme, long long capacity, double dt,
                                                   const double* X_cur_dev, const double* U0_dev,
                                                   const double* U1_dev, double* X_new_dev, const double* L, int Nz,
                                                   int nranks, int rank, const int* n_dev, int* order_dev,
                                                   int* counts_dev) {
    if (!n_dev) return fail(IBTK_LE_ERR_ARG, "null device count");
    return slab_update_partition_impl(ctx, scheme, capacity, dt, X_cur_dev, U0_dev, U1_dev, X_new_dev, L, Nz, nranks,
                                      rank, n_dev, order_dev, counts_dev);
}

extern "C" int ibtk_le_slab_migrate_pack(ibtk_le_ctx ctx, const double* rows_dev, int depth, const int* order_dev,
                                         const int* counts_dev, int send_cap, double* send_down_dev,
                                         double* send_up_dev) {
    if (!ctx || !rows_dev || !order_dev || !counts_dev || !send_down_dev || !send_up_dev)
        return fail(IBTK_LE_ERR_ARG, "migrate_pack: null argument");
    if (depth < 1 || send_cap < 0) return fail(IBTK_LE_ERR_ARG, "migrate_pack: depth >= 1, send_cap >= 0");
    if (set_device(ctx)) return IBTK_LE_ERR_DEVICE;
    HIP_TRY(launch_mig_pack(rows_dev, depth, order_dev, counts_dev, send_cap, send_down_dev, send_up_dev,
                            ctx->err.as<int>(), ctx->stream));
    return IBTK_LE_OK;
}

extern "C" int ibtk_le_slab_migrate_unpack(ibtk_le_ctx ctx, const double* rows_dev, int depth, const int* order_dev,
                                           const int* counts_dev, const int* recv_counts_dev,
                                           const double* from_down_dev, const double* from_up_dev, int send_cap,
                                           double* out_dev, int out_cap, int* n_out_dev) {
    if (!ctx || !rows_dev || !order_dev || !counts_dev || !recv_counts_dev || !from_down_dev || !from_up_dev ||
        !out_dev || !n_out_dev)
        return fail(IBTK_LE_ERR_ARG, "migrate_unpack: null argument");
    if (depth < 1 || send_cap < 0 || out_cap < 0) return fail(IBTK_LE_ERR_ARG, "migrate_unpack: bad sizes");
    if (out_dev == rows_dev) return fail(IBTK_LE_ERR_ARG, "migrate_unpack: out must not alias rows");
    if (set_device(ctx)) return IBTK_LE_ERR_DEVICE;
    HIP_TRY(launch_mig_unpack(rows_dev, depth, order_dev, counts_dev, recv_counts_dev, from_down_dev, from_up_dev,
                              send_cap, out_dev, out_cap, n_out_dev, ctx->err.as<int>(), ctx->stream));
    return IBTK_LE_OK;
}

static int slab_update_partition_impl(ibtk_le_ctx ctx, int scheme, long long M, double dt, const double* X_cur_dev,
                                      const double* U0_dev, const double* U1_dev, double* X_new_dev, const double* L,
                                      int Nz, int nranks, int rank, const int* n_dev, int* order_dev, int* counts_dev) {
    if (!ctx) return fail(IBTK_LE_ERR_ARG, "null context");
    if (scheme < IBTK_LE_EULER || scheme > IBTK_LE_TRAPEZOIDAL) return fail(IBTK_LE_ERR_ARG, "unknown update scheme");
    if (M < 0 || M >= (1LL << 31)) return fail(IBTK_LE_ERR_ARG, "marker count out of range");
    if (!L || !(L[0] > 0.0) || !(L[1] > 0.0) || !(L[2] > 0.0)) return fail(IBTK_LE_ERR_ARG, "domain lengths must be positive");
    if (nranks < 1 || rank < 0 || rank >= nranks || Nz < nranks || Nz % nranks)
        return fail(IBTK_LE_ERR_ARG, "slabs: %d ranks over %d planes (rank %d)", nranks, Nz, rank);
    if (!counts_dev) return fail(IBTK_LE_ERR_ARG, "null counts");
    HIP_TRY(hipSetDevice(ctx->device));
    if (M == 0) {
        HIP_TRY(hipMemsetAsync(counts_dev, 0, 4 * sizeof(int), ctx->stream));
        return IBTK_LE_OK;
    }
    if (!X_cur_dev || !U0_dev || !X_new_dev || !order_dev || (scheme == IBTK_LE_TRAPEZOIDAL && !U1_dev))
        return fail(IBTK_LE_ERR_ARG, "null array");
    if (X_new_dev == X_cur_dev) return fail(IBTK_LE_ERR_ARG, "X_new must not alias X_cur");
    SlabMig g;
    for (int d = 0; d < 3; ++d) g.L[d] = L[d];
    g.Nz = Nz;
    g.P = nranks;
    g.nz = Nz / nranks;
    g.rank = rank;
    g.dz = L[2] / Nz;
    g.n_dev = n_dev;
    const long nb = (long)((M + BLOCK - 1) / BLOCK);
    int rc;
    if ((rc = ctx->mig_cls.ensure((size_t)M))) return rc;
    if ((rc = ctx->mig_cnt.ensure(sizeof(int) * 8 * (size_t)nb))) return rc;
    int* bcount = ctx->mig_cnt.as<int>();
    int* boff = bcount + 4 * nb;
    size_t tb = 0;
    HIP_TRY(launch_slab_update_partition(scheme, (long)M, dt, X_cur_dev, U0_dev, U1_dev, X_new_dev, g,
                                         ctx->mig_cls.as<unsigned char>(), bcount, boff, nullptr, tb, order_dev,
                                         counts_dev, ctx->stream));
    if ((rc = ctx->temp.ensure(tb))) return rc;
    tb = ctx->temp.cap;
    HIP_TRY(launch_slab_update_partition(scheme, (long)M, dt, X_cur_dev, U0_dev, U1_dev, X_new_dev, g,
                                         ctx->mig_cls.as<unsigned char>(), bcount, boff, ctx->temp.p, tb, order_dev,
                                         counts_dev, ctx->stream));
    return IBTK_LE_OK;
}

extern "C" int ibtk_le_zero_ghosts(ibtk_le_ctx ctx, const ibtk_le_patch_geom* geom, int centering,
                                   double* const* q_dev, int q_depth) {
    return ghost_op(ctx, geom, centering, q_dev, q_depth, nullptr, 2);
}

static int index_list_impl(ibtk_le_ctx ctx, const ibtk_le_patch_geom* geom, const double* X_dev, const int* lag_dev,
                           int n_markers, int ghost, const int* periodic, int which, const int* box_lo,
                           const int* box_hi, const int* sub_lo, const int* sub_hi, int* indices_dev,
                           double* Xshift_dev, int* cells_dev, int capacity, int* count);

extern "C" int ibtk_le_periodic_index_list(ibtk_le_ctx ctx, const ibtk_le_patch_geom* geom, const double* X_dev,
                                           int n_markers, int ghost, const int* periodic, int* indices_dev,
                                           double* Xshift_dev, int capacity, int* count) {
    return index_list_impl(ctx, geom, X_dev, nullptr, n_markers, ghost, periodic, 0, nullptr, nullptr, nullptr, nullptr,
                           indices_dev, Xshift_dev, nullptr, capacity, count);
}

extern "C" int ibtk_le_index_set_list(ibtk_le_ctx ctx, const ibtk_le_patch_geom* geom, const double* X_dev,
                                      const int* lag_dev, int n_markers, int ghost, const int* periodic, int which,
                                      int* indices_dev, double* Xshift_dev, int capacity, int* count) {
    if (which < 0 || which > 2) return fail(IBTK_LE_ERR_ARG, "which: 0 all, 1 interior, 2 ghost");
    return index_list_impl(ctx, geom, X_dev, lag_dev, n_markers, ghost, periodic, which, nullptr, nullptr, nullptr,
                           nullptr, indices_dev, Xshift_dev, nullptr, capacity, count);
}

extern "C" int ibtk_le_index_set_box_list(ibtk_le_ctx ctx, const ibtk_le_patch_geom* geom, const double* X_dev,
                                          const int* lag_dev, int n_markers, int ghost, const int* periodic,
                                          const int* box_lo, const int* box_hi, int* indices_dev, double* Xshift_dev,
                                          int* cells_dev, int capacity, int* count) {
    if (!box_lo || !box_hi) return fail(IBTK_LE_ERR_ARG, "null box");
    return index_list_impl(ctx, geom, X_dev, lag_dev, n_markers, ghost, periodic, 0, nullptr, nullptr, box_lo, box_hi,
                           indices_dev, Xshift_dev, cells_dev, capacity, count);
}

extern "C" int ibtk_le_box_index_list(ibtk_le_ctx ctx, const ibtk_le_patch_geom* geom, const double* X_dev,
                                      int n_markers, const int* box_lo, const int* box_hi, int* indices_dev,
                                      int capacity, int* count) {
    if (!box_lo || !box_hi) return fail(IBTK_LE_ERR_ARG, "null box");
    return index_list_impl(ctx, geom, X_dev, nullptr, n_markers, 0, nullptr, 0, box_lo, box_hi, nullptr, nullptr,
                           indices_dev, nullptr, nullptr, capacity, count);
}

// Stable compaction of a list by flags (exclusive scan, one host sync for the count).
static int compact_by_flags(ibtk_le_ctx ctx, int ndim, int n, const int* flag, const int* idx, const double* xs,
                            const int* cells, int* idx_out, double* xs_out, int* cells_out, int capacity,
                            int* count) {
    const hipStream_t s = ctx->stream;
    int rc;
    if ((rc = ctx->lst_flag.ensure(sizeof(int) * (size_t)n))) return rc;
    int* pos = ctx->lst_flag.as<int>();
    size_t tb = 0;
    HIP_TRY(launch_scan(nullptr, tb, flag, pos, n, s));
    if ((rc = ctx->temp.ensure(tb))) return rc;
    tb = ctx->temp.cap;
    HIP_TRY(launch_scan(ctx->temp.p, tb, flag, pos, n, s));
    int last[2] = {0, 0};
    HIP_TRY(hipMemcpyAsync(&last[0], pos + n - 1, sizeof(int), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(&last[1], flag + n - 1, sizeof(int), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    *count = last[0] + last[1];
    if (*count > capacity || (*count > 0 && !idx_out))
        return fail(IBTK_LE_ERR_ARG, "index list needs %d entries, capacity %d", *count, capacity);
    HIP_TRY(launch_compact_list(flag, pos, idx, xs, cells, ndim, n, idx_out, xs_out, cells_out, s));
    return IBTK_LE_OK;
}

extern "C" int ibtk_le_list_in_box(ibtk_le_ctx ctx, int ndim, const int* cells_dev, const int* indices_dev,
                                   const double* Xshift_dev, int n, const int* box_lo, const int* box_hi,
                                   int* indices_out, double* Xshift_out, int capacity, int* count) {
    if (!ctx || !count || !box_lo || !box_hi) return fail(IBTK_LE_ERR_ARG, "null argument");
    if (ndim != 2 && ndim != 3) return fail(IBTK_LE_ERR_ARG, "ndim must be 2 or 3");
    if (n < 0) return fail(IBTK_LE_ERR_ARG, "negative size");
    *count = 0;
    if (n == 0) return IBTK_LE_OK;
    if (!cells_dev || !indices_dev) return fail(IBTK_LE_ERR_ARG, "null list");
    if (set_device(ctx)) return IBTK_LE_ERR_DEVICE;
    int rc;
    if ((rc = ctx->lst_perm.ensure(sizeof(int) * (size_t)n))) return rc;
    HIP_TRY(launch_in_box_flags(cells_dev, ndim, n, box_lo, box_hi, ctx->lst_perm.as<int>(), ctx->stream));
    return compact_by_flags(ctx, ndim, n, ctx->lst_perm.as<int>(), indices_dev, Xshift_dev, nullptr, indices_out,
                            Xshift_dev ? Xshift_out : nullptr, nullptr, capacity, count);
}

static ImageDesc image_desc(const ibtk_le_patch_geom* geom, int ghost) {
    ImageDesc d;
    std::memset(&d, 0, sizeof(d));
    d.ndim = geom->ndim;
    d.ghost = ghost;
    for (int k = 0; k < geom->ndim; ++k) {
        d.xlo[k] = geom->x_lower[k];
        d.xup[k] = geom->x_upper[k];
        d.dx[k] = geom->dx[k];
        d.ilo[k] = geom->ilower[k];
        d.ihi[k] = geom->iupper[k];
    }
    return d;
}

// Two stable radix passes: by the Lagrangian index (lag, or the marker index
// idx[i] / i when lag is null), then by the cell key; perm[i] = the entry of
// rank i.  The sorted keys are left in kbuf's upper half.
static int sort_cell_lag(ibtk_le_ctx ctx, const unsigned* cell_keys, const int* idx, const int* lag, int n,
                         unsigned long long key_end, int* perm, DevBuf& kbuf, DevBuf& vbuf) {
    const hipStream_t s = ctx->stream;
    int rc;
    if ((rc = kbuf.ensure(2 * sizeof(unsigned) * (size_t)n))) return rc;
    if ((rc = vbuf.ensure(sizeof(int) * (size_t)n))) return rc;
    unsigned* k0 = kbuf.as<unsigned>();
    unsigned* k1 = k0 + n;
    int* v0 = vbuf.as<int>();
    size_t tb = 0;
    HIP_TRY(launch_sort(nullptr, tb, k0, k1, v0, perm, n, 32, s));
    if ((rc = ctx->temp.ensure(tb))) return rc;
    tb = ctx->temp.cap;
    HIP_TRY(launch_iota(v0, n, s));
    if (lag) {  // pass 1 (entries are generated in marker order: the marker index needs no pass)
        HIP_TRY(launch_perm_keys(0, nullptr, idx, lag, nullptr, n, k0, s));
        HIP_TRY(launch_sort(ctx->temp.p, tb, k0, k1, v0, perm, n, 32, s));
        HIP_TRY(hipMemcpyAsync(v0, perm, sizeof(int) * (size_t)n, hipMemcpyDeviceToDevice, s));
    }
    HIP_TRY(launch_perm_keys(1, v0, nullptr, nullptr, cell_keys, n, k0, s));
    int end_bit = 1;
    while (end_bit < 32 && (1ull << end_bit) <= key_end) ++end_bit;
    HIP_TRY(launch_sort(ctx->temp.p, tb, k0, k1, v0, perm, n, end_bit, s));
    return IBTK_LE_OK;
}

// The index lists of one patch (LIndexSetData::cacheLocalIndices, LIndexSetData.cpp:
// 83-169, and LEInteractor::buildLocalIndices' box branch, LEInteractor.cpp:3070-3106):
// every marker of the patch box at its cell and its periodic images at theirs, the
// entries in the ghost box's cell iteration order, each cell's set sorted by
// Lagrangian index and, when Lagrangian indices are given, uniqued
// (LDataManager.cpp:1487-1493: the lowest marker index of equal ones is kept).
// which selects interior / ghost cells, [sub_lo, sub_hi] any box of cells.  box_lo
// instead: the X-only box filter (LEInteractor.cpp:3110-3139, marker order).
static int index_list_impl(ibtk_le_ctx ctx, const ibtk_le_patch_geom* geom, const double* X_dev, const int* lag_dev,
                           int n_markers, int ghost, const int* periodic, int which, const int* box_lo,
                           const int* box_hi, const int* sub_lo, const int* sub_hi, int* indices_dev,
                           double* Xshift_dev, int* cells_dev, int capacity, int* count) {
    if (!ctx || !count) return fail(IBTK_LE_ERR_ARG, "null argument");
    if (int rc = check_geom(geom)) return rc;
    if (n_markers < 0 || ghost < 0) return fail(IBTK_LE_ERR_ARG, "negative size");
    if (set_device(ctx)) return IBTK_LE_ERR_DEVICE;
    *count = 0;
    if (n_markers == 0) return IBTK_LE_OK;
    ImageDesc d = image_desc(geom, ghost);
    d.which = which;
    unsigned long long gcells = 1;
    for (int k = 0; k < geom->ndim; ++k) {
        d.periodic[k] = periodic ? periodic[k] : 1;
        if (box_lo) {
            d.filter = 1;
            d.flo[k] = box_lo[k];
            d.fhi[k] = box_hi[k];
        }
        if (sub_lo) {
            d.sub = 1;
            d.slo[k] = sub_lo[k];
            d.shi[k] = sub_hi[k];
        }
        gcells *= (unsigned long long)(geom->iupper[k] - geom->ilower[k] + 1 + 2 * ghost);
    }
    if (gcells >= 0xffffffffull) return fail(IBTK_LE_ERR_RANGE, "ghost box has %llu cells", gcells);
    int rc;
    if ((rc = ctx->counts.ensure(sizeof(int) * (size_t)n_markers))) return rc;
    if ((rc = ctx->offsets.ensure(sizeof(int) * (size_t)n_markers))) return rc;
    const hipStream_t s = ctx->stream;
    HIP_TRY(launch_image_count(d, X_dev, n_markers, ctx->counts.as<int>(), s));
    size_t tb = 0;
    HIP_TRY(launch_scan(nullptr, tb, ctx->counts.as<int>(), ctx->offsets.as<int>(), n_markers, s));
    if ((rc = ctx->temp.ensure(tb))) return rc;
    tb = ctx->temp.cap;
    HIP_TRY(launch_scan(ctx->temp.p, tb, ctx->counts.as<int>(), ctx->offsets.as<int>(), n_markers, s));
    int last[2] = {0, 0};
    HIP_TRY(hipMemcpyAsync(&last[0], ctx->offsets.as<int>() + n_markers - 1, sizeof(int), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(&last[1], ctx->counts.as<int>() + n_markers - 1, sizeof(int), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    const int total = last[0] + last[1];
    *count = total;
    if (box_lo) {  // LEInteractor.cpp:3110-3139: marker order
        if (total > capacity || !indices_dev)
            return fail(IBTK_LE_ERR_ARG, "index list needs %d entries, capacity %d", total, capacity);
        HIP_TRY(launch_image_write(d, X_dev, n_markers, ctx->offsets.as<int>(), indices_dev, Xshift_dev, nullptr,
                                   nullptr, capacity, s));
        return IBTK_LE_OK;
    }
    if (total == 0) return IBTK_LE_OK;
    if (!lag_dev && (total > capacity || !indices_dev || !Xshift_dev))
        return fail(IBTK_LE_ERR_ARG, "index list needs %d entries, capacity %d", total, capacity);
    // entries in marker order into scratch, then the reference's order: cells of
    // the ghost box in iteration order (x fastest), Lagrangian index within a cell
    const size_t nd = (size_t)geom->ndim;
    if ((rc = ctx->lst_idx.ensure(sizeof(int) * (size_t)total))) return rc;
    if ((rc = ctx->lst_xs.ensure(sizeof(double) * nd * (size_t)total))) return rc;
    if ((rc = ctx->lst_key.ensure(sizeof(unsigned) * (size_t)total))) return rc;
    if ((rc = ctx->lst_cell.ensure(sizeof(int) * nd * (size_t)total))) return rc;
    if ((rc = ctx->lst_perm.ensure(sizeof(int) * (size_t)total))) return rc;
    HIP_TRY(launch_image_write(d, X_dev, n_markers, ctx->offsets.as<int>(), ctx->lst_idx.as<int>(),
                               ctx->lst_xs.as<double>(), ctx->lst_key.as<unsigned>(), ctx->lst_cell.as<int>(), total,
                               s));
    if ((rc = sort_cell_lag(ctx, ctx->lst_key.as<unsigned>(), ctx->lst_idx.as<int>(), lag_dev, total, gcells,
                            ctx->lst_perm.as<int>(), ctx->keys_in, ctx->vals_in)))
        return rc;
    if (!lag_dev) {  // markers by index: no two entries of one cell share one
        HIP_TRY(launch_perm_list(ctx->lst_perm.as<int>(), ctx->lst_idx.as<int>(), ctx->lst_xs.as<double>(),
                                 ctx->lst_cell.as<int>(), geom->ndim, total, indices_dev, Xshift_dev, cells_dev, s));
        return IBTK_LE_OK;
    }
    // the sorted list into scratch, then the first of every (cell, Lagrangian index)
    if ((rc = ctx->lst2_idx.ensure(sizeof(int) * (size_t)total))) return rc;
    if ((rc = ctx->lst2_xs.ensure(sizeof(double) * nd * (size_t)total))) return rc;
    if ((rc = ctx->lst2_cell.ensure(sizeof(int) * nd * (size_t)total))) return rc;
    HIP_TRY(launch_perm_list(ctx->lst_perm.as<int>(), ctx->lst_idx.as<int>(), ctx->lst_xs.as<double>(),
                             ctx->lst_cell.as<int>(), geom->ndim, total, ctx->lst2_idx.as<int>(),
                             ctx->lst2_xs.as<double>(), ctx->lst2_cell.as<int>(), s));
    const unsigned* skeys = ctx->keys_in.as<unsigned>() + total;  // sorted keys (sort_cell_lag)
    int* flag = ctx->lst_perm.as<int>();                           // the permutation is spent
    HIP_TRY(launch_unique_flags(skeys, ctx->lst2_idx.as<int>(), lag_dev, total, flag, s));
    return compact_by_flags(ctx, geom->ndim, total, flag, ctx->lst2_idx.as<int>(), ctx->lst2_xs.as<double>(),
                            ctx->lst2_cell.as<int>(), indices_dev, Xshift_dev, cells_dev, capacity, count);
}

// LDataManager::computeNodeDistribution (LDataManager.cpp:2839-3027) for one
// patch whose LNodeSetData has `ghost` ghost cells: the local nodes -- markers
// whose getCellIndex cell is in the patch box -- first, cell by cell in box
// order (x fastest), each cell's set in Lagrangian-index order and uniqued
// (LDataManager.cpp:1487-1493); then the nonlocal nodes of the ghost cells in
// ghost-box order.  order_dev[i] = the input index of the node numbered i.
extern "C" int ibtk_le_node_distribution(ibtk_le_ctx ctx, const ibtk_le_patch_geom* geom, const double* X_dev,
                                         const int* lag_dev, int n_markers, int ghost, int* order_dev, int* n_local,
                                         int* n_nonlocal) {
    if (!ctx || !n_local || !n_nonlocal) return fail(IBTK_LE_ERR_ARG, "null argument");
    if (int rc = check_geom(geom)) return rc;
    if (n_markers < 0 || ghost < 0) return fail(IBTK_LE_ERR_ARG, "negative size");
    if (n_markers > 0 && (!X_dev || !order_dev)) return fail(IBTK_LE_ERR_ARG, "null array");
    *n_local = *n_nonlocal = 0;
    if (n_markers == 0) return IBTK_LE_OK;
    unsigned long long ncell = 1, gcells = 1;
    for (int k = 0; k < geom->ndim; ++k) {
        ncell *= (unsigned long long)(geom->iupper[k] - geom->ilower[k] + 1);
        gcells *= (unsigned long long)(geom->iupper[k] - geom->ilower[k] + 1 + 2 * ghost);
    }
    if (ncell + gcells >= 0xffffffffull) return fail(IBTK_LE_ERR_RANGE, "patch too large for 32-bit cell keys");
    if (set_device(ctx)) return IBTK_LE_ERR_DEVICE;
    const ImageDesc d = image_desc(geom, ghost);
    const hipStream_t s = ctx->stream;
    const int n = n_markers;
    int rc;
    if ((rc = ctx->lst_key.ensure(sizeof(unsigned) * (size_t)n))) return rc;
    if ((rc = ctx->lst_perm.ensure(sizeof(int) * (size_t)n))) return rc;
    if ((rc = ctx->lst_idx.ensure(2 * sizeof(int) * (size_t)n))) return rc;  // flags | positions
    if ((rc = ctx->counts.ensure(2 * sizeof(int)))) return rc;
    HIP_TRY(launch_node_keys(d, X_dev, n, ctx->lst_key.as<unsigned>(), s));
    if ((rc = sort_cell_lag(ctx, ctx->lst_key.as<unsigned>(), nullptr, lag_dev, n, 0xffffffffull,
                            ctx->lst_perm.as<int>(), ctx->keys_in, ctx->vals_in)))
        return rc;
    const unsigned* skeys = ctx->keys_in.as<unsigned>() + n;  // sorted keys (sort_cell_lag)
    int* flag = ctx->lst_idx.as<int>();
    int* pos = flag + n;
    HIP_TRY(launch_unique_flags(skeys, ctx->lst_perm.as<int>(), lag_dev, n, flag, s));
    size_t tb = 0;
    HIP_TRY(launch_scan(nullptr, tb, flag, pos, n, s));
    if ((rc = ctx->temp.ensure(tb))) return rc;
    tb = ctx->temp.cap;
    HIP_TRY(launch_scan(ctx->temp.p, tb, flag, pos, n, s));
    HIP_TRY(hipMemsetAsync(ctx->counts.p, 0, 2 * sizeof(int), s));
    HIP_TRY(launch_compact(ctx->lst_perm.as<int>(), flag, pos, skeys, (unsigned)ncell, (unsigned)(ncell + gcells), n,
                           order_dev, ctx->counts.as<int>(), s));
    int cnt[2] = {0, 0};
    HIP_TRY(hipMemcpyAsync(cnt, ctx->counts.p, 2 * sizeof(int), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    *n_local = cnt[0];
    *n_nonlocal = cnt[1];
    return IBTK_LE_OK;
}

// Stable sort of (keys, vals) on the context stream: out_keys/out_vals may be
// scratch of the caller; uses ctx->temp.
static int sort_pairs(ibtk_le_ctx ctx, const unsigned* kin, unsigned* kout, const int* vin, int* vout, int n,
                      int end_bit) {
    size_t tb = 0;
    HIP_TRY(launch_sort(nullptr, tb, kin, kout, vin, vout, n, end_bit, ctx->stream));
    if (int rc = ctx->temp.ensure(tb)) return rc;
    tb = ctx->temp.cap;
    HIP_TRY(launch_sort(ctx->temp.p, tb, kin, kout, vin, vout, n, end_bit, ctx->stream));
    return IBTK_LE_OK;
}

// bytes of device memory to host memory after the stream's work so far: one copy through the
// context's pinned staging, then a wait on the stream
static int d2h_sync(ibtk_le_ctx ctx, void* host, const void* dev, size_t bytes) {
    if (ctx->hstage_cap < bytes) {
        if (ctx->hstage) HIP_TRY(hipHostFree(ctx->hstage));
        ctx->hstage = nullptr;
        ctx->hstage_cap = 0;
        const size_t cap = std::max<size_t>(bytes, 4096);
        HIP_TRY(hipHostMalloc(&ctx->hstage, cap, hipHostMallocDefault));
        ctx->hstage_cap = cap;
    }
    HIP_TRY(hipMemcpyAsync(ctx->hstage, dev, bytes, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    std::memcpy(host, ctx->hstage, bytes);
    return IBTK_LE_OK;
}

// A level of equal patches aligned to one tiling of the domain [dom_lo, dom_hi]: its
// numbering frame (LevelNum) and the tile -> patch table (-1: no local patch).
static int make_level_num(int npatch, const ibtk_le_patch_geom* geoms, const int* dom_lo, const int* dom_hi,
                          const int* periodic, int ghost, LevelNum& L, std::vector<int>& tab) {
    if (!geoms || !dom_lo || !dom_hi) return fail(IBTK_LE_ERR_ARG, "null argument");
    if (npatch < 1 || ghost < 0) return fail(IBTK_LE_ERR_ARG, "bad sizes");
    const int nd = geoms[0].ndim;
    std::memset(&L, 0, sizeof(L));
    L.ndim = nd;
    L.g = ghost;
    for (int q = 0; q < npatch; ++q) {
        if (int rc = check_geom(&geoms[q])) return rc;
        if (geoms[q].ndim != nd) return fail(IBTK_LE_ERR_ARG, "patches of different dimension");
        for (int k = 0; k < nd; ++k) {
            const int nk = geoms[q].iupper[k] - geoms[q].ilower[k] + 1;
            if (q == 0) {
                L.n[k] = nk;
                L.rn[k] = 1.0f / (float)nk;
                L.org[k] = geoms[0].ilower[k];
                L.dx[k] = geoms[0].dx[k];
            }
            if (nk != L.n[k] || geoms[q].dx[k] != L.dx[k])
                return fail(IBTK_LE_ERR_ARG, "level numbering needs patches of one size and spacing");
            L.org[k] = std::min(L.org[k], geoms[q].ilower[k]);
        }
    }
    long long ntab = 1, pcells = 1, gcells = 1;
    for (int k = 0; k < nd; ++k) {
        int tmax = 0;
        for (int q = 0; q < npatch; ++q) {
            if ((geoms[q].ilower[k] - L.org[k]) % L.n[k])
                return fail(IBTK_LE_ERR_ARG, "patch %d is not aligned to the level's tiling", q);
            tmax = std::max(tmax, (geoms[q].ilower[k] - L.org[k]) / L.n[k]);
        }
        L.nt[k] = tmax + 1;
        ntab *= L.nt[k];
        pcells *= L.n[k];
        gcells *= L.n[k] + 2 * ghost;
        L.dom_lo[k] = dom_lo[k];
        L.dom_hi[k] = dom_hi[k];
        L.periodic[k] = periodic ? periodic[k] != 0 : 1;
        L.xlo[k] = geoms[0].x_lower[k] - (double)(geoms[0].ilower[k] - dom_lo[k]) * L.dx[k];
        L.xup[k] = L.xlo[k] + (double)(dom_hi[k] - dom_lo[k] + 1) * L.dx[k];
    }
    if ((long long)npatch * pcells >= 0xffffffffLL || (long long)npatch * gcells >= 0xfffffffeLL)
        return fail(IBTK_LE_ERR_RANGE, "level too large for 32-bit node keys");
    tab.assign((size_t)ntab, -1);
    for (int q = 0; q < npatch; ++q) {
        long long lin = 0, str = 1;
        for (int k = 0; k < nd; ++k) {
            lin += (long long)((geoms[q].ilower[k] - L.org[k]) / L.n[k]) * str;
            str *= L.nt[k];
        }
        if (tab[(size_t)lin] >= 0) return fail(IBTK_LE_ERR_ARG, "patches %d and %d overlap", tab[(size_t)lin], q);
        tab[(size_t)lin] = q;
    }
    return IBTK_LE_OK;
}

// LDataManager::computeNodeDistribution (LDataManager.cpp:2874-2947) over the local
// patches of a level (geoms[q], q in PatchLevel order): the local nodes patch by
// patch (data_begin(patch_box): box cells, x fastest; each cell's set by Lagrangian
// index, uniqued, :1487-1493), then the nonlocal ones -- nodes of the patches' ghost
// cells whose Lagrangian index no local node has -- each at its first sighting
// (patches in order, a patch's ghost cells in ghost-box order).  The patches are equal
// boxes aligned to one tiling of the domain [dom_lo, dom_hi] (periodic images across
// its periodic sides, the index data's periodic ghost fill).
extern "C" int ibtk_le_level_node_distribution(ibtk_le_ctx ctx, int npatch, const ibtk_le_patch_geom* geoms,
                                               const int* dom_lo, const int* dom_hi, const int* periodic,
                                               const double* X_dev, const int* lag_dev, int n_markers, int ghost,
                                               int* order_dev, int* n_local, int* n_nonlocal) {
    if (!ctx || !n_local || !n_nonlocal) return fail(IBTK_LE_ERR_ARG, "null argument");
    if (n_markers < 0) return fail(IBTK_LE_ERR_ARG, "bad sizes");
    *n_local = *n_nonlocal = 0;
    LevelNum L;
    std::vector<int> tab;
    if (int rc = make_level_num(npatch, geoms, dom_lo, dom_hi, periodic, ghost, L, tab)) return rc;
    if (n_markers == 0) return IBTK_LE_OK;
    if (!X_dev || !order_dev) return fail(IBTK_LE_ERR_ARG, "null array");
    if (set_device(ctx)) return IBTK_LE_ERR_DEVICE;
    const hipStream_t s = ctx->stream;
    const int n = n_markers;
    int rc;
    if ((rc = ctx->num_tab.ensure(sizeof(int) * tab.size()))) return rc;
    if ((rc = ctx->num_lkey.ensure(sizeof(unsigned) * (size_t)n))) return rc;
    if ((rc = ctx->num_ckey.ensure(sizeof(unsigned) * (size_t)n))) return rc;
    if ((rc = ctx->lst_perm.ensure(sizeof(int) * (size_t)n))) return rc;
    if ((rc = ctx->lst2_idx.ensure(2 * sizeof(int) * (size_t)n))) return rc;
    if ((rc = ctx->lst_key.ensure(2 * sizeof(unsigned) * (size_t)n))) return rc;
    HIP_TRY(hipMemcpyAsync(ctx->num_tab.p, tab.data(), sizeof(int) * tab.size(), hipMemcpyHostToDevice, s));
    unsigned* lkey = ctx->num_lkey.as<unsigned>();
    unsigned* ckey = ctx->num_ckey.as<unsigned>();
    HIP_TRY(launch_level_node_keys(L, ctx->num_tab.as<int>(), X_dev, n, lkey, ckey, s));
    // local nodes: by (patch, cell, Lagrangian index), the first of each (cell, index)
    int* perm = ctx->lst_perm.as<int>();
    if ((rc = sort_cell_lag(ctx, lkey, nullptr, lag_dev, n, 0xffffffffull, perm, ctx->keys_in, ctx->vals_in)))
        return rc;
    int* flag = ctx->lst2_idx.as<int>();
    int* spare = flag + n;
    HIP_TRY(launch_unique_flags(ctx->keys_in.as<unsigned>() + n, perm, lag_dev, n, flag, s));
    int cnt = 0;
    if ((rc = compact_by_flags(ctx, 1, n, flag, perm, nullptr, nullptr, order_dev, nullptr, nullptr, n, &cnt)))
        return rc;
    const int nl = cnt;
    if (ghost == 0) {  // no ghost cells: every marker outside the local patches is nobody's node here
        *n_local = nl;
        return IBTK_LE_OK;
    }
    // nonlocal nodes: the markers by (Lagrangian index, first sighting), the head of
    // every index run whose run holds no local node, then by first sighting
    unsigned* k0 = ctx->lst_key.as<unsigned>();
    unsigned* k1 = k0 + n;
    int* v0 = ctx->vals_in.as<int>();
    HIP_TRY(launch_iota(v0, n, s));
    if ((rc = sort_pairs(ctx, ckey, k1, v0, perm, n, 32))) return rc;
    HIP_TRY(launch_perm_keys(0, perm, nullptr, lag_dev, nullptr, n, k0, s));
    if ((rc = sort_pairs(ctx, k0, k1, perm, spare, n, 32))) return rc;  // spare: markers by (lag, ckey)
    HIP_TRY(launch_take_keys(ckey, spare, n, k0, s));
    HIP_TRY(launch_nonlocal_flags(k0, spare, lag_dev, n, flag, s));
    if ((rc = compact_by_flags(ctx, 1, n, flag, spare, nullptr, nullptr, perm, nullptr, nullptr, n, &cnt))) return rc;
    const int nn = cnt;
    if (nn > 0) {
        HIP_TRY(launch_take_keys(ckey, perm, nn, k0, s));
        if ((rc = sort_pairs(ctx, k0, k1, perm, order_dev + nl, nn, 32))) return rc;
    }
    HIP_TRY(hipStreamSynchronize(s));
    *n_local = nl;
    *n_nonlocal = nn;
    return IBTK_LE_OK;
}

// LIndexSetData::cacheLocalIndices (LIndexSetData.cpp:83-169) for every local patch of a
// level in one pass -- the per-patch lists LDataManager::spread / interp hand LEInteractor
// (LDataManager.cpp:634-654, 763-807): the interior lists (markers whose getCellIndex cell
// is in the patch box) and the ghost-box lists (markers and their periodic images whose
// cell is in the patch's ghost box, with their shifts), patch by patch, each patch's
// entries in its box's (ghost box's) cell order, x fastest, a cell's markers by index --
// the order ibtk_le_periodic_index_list gives one patch -- or (order 1) in marker order.
// Keys per marker, a stable device radix sort by (patch, cell) or by patch alone (fewer
// passes), the patch offsets by binary search in the sorted keys.
extern "C" int ibtk_le_level_index_lists(ibtk_le_ctx ctx, int npatch, const ibtk_le_patch_geom* geoms,
                                         const int* dom_lo, const int* dom_hi, const int* periodic,
                                         const double* X_dev, int n_markers, int ghost, int order, int* interior_dev,
                                         int interior_cap, int* interior_off, int* ghost_dev, double* Xshift_dev,
                                         int ghost_cap, int* ghost_off) {
    if (!ctx || !interior_off || !ghost_off) return fail(IBTK_LE_ERR_ARG, "null argument");
    if (order != 0 && order != 1) return fail(IBTK_LE_ERR_ARG, "level_index_lists: order 0 (cells) or 1 (markers)");
    if (n_markers < 0 || interior_cap < 0 || ghost_cap < 0) return fail(IBTK_LE_ERR_ARG, "bad sizes");
    LevelNum L;
    std::vector<int> tab;
    if (int rc = make_level_num(npatch, geoms, dom_lo, dom_hi, periodic, ghost, L, tab)) return rc;
    for (int q = 0; q <= npatch; ++q) interior_off[q] = ghost_off[q] = 0;
    const int n = n_markers;
    if (n == 0) return IBTK_LE_OK;
    if (!X_dev) return fail(IBTK_LE_ERR_ARG, "null X");
    unsigned pcells = 1, gcells = 1;
    for (int k = 0; k < L.ndim; ++k) {
        pcells *= (unsigned)L.n[k];
        gcells *= (unsigned)(L.n[k] + 2 * ghost);
    }
    const int bypatch = order;
    int pbits = 1;  // bits of the patch keys 0 .. npatch
    while ((1LL << pbits) <= (long long)npatch) ++pbits;
    const int kbits = bypatch ? pbits : 32;
    if (bypatch) pcells = gcells = 1;  // (the offsets' key stride)
    if (set_device(ctx)) return IBTK_LE_ERR_DEVICE;
    const hipStream_t s = ctx->stream;
    int rc;
    if ((rc = ctx->num_tab.ensure(sizeof(int) * tab.size()))) return rc;
    if ((rc = ctx->ll_cnt.ensure(sizeof(int) * (size_t)(n + 1)))) return rc;
    if ((rc = ctx->ll_off.ensure(sizeof(int) * (size_t)(n + 1)))) return rc;
    if ((rc = ctx->ll_key.ensure(sizeof(unsigned) * (size_t)n))) return rc;
    if ((rc = ctx->ll_key2.ensure(sizeof(unsigned) * (size_t)n))) return rc;
    if ((rc = ctx->ll_id.ensure(sizeof(int) * (size_t)n))) return rc;
    if ((rc = ctx->ll_id2.ensure(sizeof(int) * (size_t)n))) return rc;
    // the patch offsets (npatch + 1 ints), the ghost-box entries' 32-bit total, then their
    // 64-bit total: read back in one copy
    const size_t sum_at = ((sizeof(int) * (size_t)(npatch + 2)) + 7) / 8 * 8;
    if ((rc = ctx->counts.ensure(sum_at + sizeof(unsigned long long)))) return rc;
    unsigned long long* const total64_dev = reinterpret_cast<unsigned long long*>(ctx->counts.as<char>() + sum_at);
    HIP_TRY(hipMemcpyAsync(ctx->num_tab.p, tab.data(), sizeof(int) * tab.size(), hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemsetAsync(ctx->ll_cnt.as<int>() + n, 0, sizeof(int), s));
    HIP_TRY(hipMemsetAsync(total64_dev, 0, sizeof(unsigned long long), s));
    HIP_TRY(launch_level_list_keys(L, ctx->num_tab.as<int>(), X_dev, n, ctx->ll_key.as<unsigned>(),
                                   ctx->ll_cnt.as<int>(), bypatch, npatch, s));
    // A marker may have many ghost-box entries (its images near the domain's faces, each in
    // the ghost boxes of several small patches): where n times the most a marker can have
    // reaches 2^31, the entries' 32-bit scan below is checked against their sum in 64 bits,
    // and a level with 2^31 entries or more is refused (advisor, round 5)
    // per dim: 2 images (3 in a domain no wider than 2 g), each in the ghost boxes of at most
    // 2 g / n + 2 tiles
    long long per_max = 1;
    for (int k = 0; k < L.ndim; ++k) {
        const long long images = (L.dom_hi[k] - L.dom_lo[k] + 1 > 2LL * ghost) ? 2 : 3;
        per_max *= images * (2LL * ghost / std::max(1, L.n[k]) + 2);
    }
    const bool check64 = (long long)n * per_max >= (1LL << 31);
    if (check64) HIP_TRY(launch_sum64(ctx->ll_cnt.as<int>(), n, total64_dev, s));
    if ((rc = scan_excl(ctx, ctx->ll_cnt.as<int>(), ctx->ll_off.as<int>(), n + 1))) return rc;
    // interior: markers by (patch, cell), stable
    HIP_TRY(launch_iota(ctx->ll_id.as<int>(), n, s));
    if ((rc = sort_pairs(ctx, ctx->ll_key.as<unsigned>(), ctx->ll_key2.as<unsigned>(), ctx->ll_id.as<int>(),
                         ctx->ll_id2.as<int>(), n, kbits)))
        return rc;
    HIP_TRY(launch_key_offsets(ctx->ll_key2.as<unsigned>(), n, pcells, npatch, ctx->counts.as<int>(), s));
    HIP_TRY(hipMemcpyAsync(ctx->counts.as<int>() + npatch + 1, ctx->ll_off.as<int>() + n, sizeof(int),
                           hipMemcpyDeviceToDevice, s));
    std::vector<char> back(sum_at + sizeof(unsigned long long));
    if ((rc = d2h_sync(ctx, back.data(), ctx->counts.p, back.size()))) return rc;
    std::memcpy(interior_off, back.data(), sizeof(int) * (size_t)(npatch + 1));
    int total = 0;
    unsigned long long total64 = 0;
    std::memcpy(&total, back.data() + sizeof(int) * (size_t)(npatch + 1), sizeof(int));
    std::memcpy(&total64, back.data() + sum_at, sizeof(total64));
    if (!check64) total64 = (unsigned long long)(unsigned)total;
    if (total64 >= (1ULL << 31) || (unsigned long long)total != total64)
        return fail(IBTK_LE_ERR_RANGE, "level_index_lists: %llu ghost-box entries (2^31 or more)", total64);
    const int nint = interior_off[npatch];
    bool short_cap = nint > interior_cap;
    if (nint > 0 && !short_cap) {
        if (!interior_dev) return fail(IBTK_LE_ERR_ARG, "null interior list");
        HIP_TRY(hipMemcpyAsync(interior_dev, ctx->ll_id2.p, sizeof(int) * (size_t)nint, hipMemcpyDeviceToDevice, s));
    }
    // ghost boxes: entries per marker in marker order, then by (patch, cell), stable
    if (total > 0) {
        for (DevBuf* b : {&ctx->ll_src, &ctx->ll_img})
            if ((rc = b->ensure(sizeof(int) * (size_t)total))) return rc;
        if ((size_t)total > (size_t)n) {  // the interior's scratch reused, grown to the entries
            for (DevBuf* b : {&ctx->ll_key, &ctx->ll_key2, &ctx->ll_id, &ctx->ll_id2})
                if ((rc = b->ensure(sizeof(int) * (size_t)total))) return rc;
        }
        HIP_TRY(launch_level_list_write(L, ctx->num_tab.as<int>(), X_dev, n, ctx->ll_off.as<int>(),
                                        ctx->ll_key.as<unsigned>(), ctx->ll_id.as<int>(), ctx->ll_src.as<int>(),
                                        ctx->ll_img.as<int>(), bypatch, s));
        if ((rc = sort_pairs(ctx, ctx->ll_key.as<unsigned>(), ctx->ll_key2.as<unsigned>(), ctx->ll_id.as<int>(),
                             ctx->ll_id2.as<int>(), total, kbits)))
            return rc;
        HIP_TRY(launch_key_offsets(ctx->ll_key2.as<unsigned>(), total, gcells, npatch, ctx->counts.as<int>(), s));
        if ((rc = d2h_sync(ctx, ghost_off, ctx->counts.p, sizeof(int) * (size_t)(npatch + 1)))) return rc;
        if (total <= ghost_cap) {
            if (!ghost_dev) return fail(IBTK_LE_ERR_ARG, "null ghost-box list");
            HIP_TRY(launch_level_list_out(L, ctx->ll_id2.as<int>(), ctx->ll_src.as<int>(), ctx->ll_img.as<int>(), total,
                                          ghost_dev, Xshift_dev, s));
        } else {
            short_cap = true;
        }
    }
    // (no wait for the lists' write: the offsets are on the host already, the lists follow
    // on the stream, and the caller's next launches queue behind them)
    if (short_cap)
        return fail(IBTK_LE_ERR_ARG, "level_index_lists: %d interior / %d ghost-box entries exceed the capacities %d / %d",
                    nint, total, interior_cap, ghost_cap);
    return IBTK_LE_OK;
}

// beginDataRedistribution's wrap of the positions into the periodic domain
// (LDataManager.cpp:1385-1399), in place: per periodic dim, += / -= the domain length
// while outside [x_lower, x_upper), then clamped into [x_lower, x_upper - eps].
extern "C" int ibtk_le_wrap_positions(ibtk_le_ctx ctx, int ndim, long long n, double* X_dev, const double* x_lower,
                                      const double* x_upper, const int* periodic) {
    if (!ctx || !x_lower || !x_upper) return fail(IBTK_LE_ERR_ARG, "null argument");
    if (ndim < 1 || ndim > 3 || n < 0) return fail(IBTK_LE_ERR_ARG, "bad sizes");
    if (n == 0) return IBTK_LE_OK;
    if (!X_dev) return fail(IBTK_LE_ERR_ARG, "null X");
    WrapBox w;
    for (int d = 0; d < 3; ++d) {
        w.lo[d] = d < ndim ? x_lower[d] : 0.0;
        w.hi[d] = d < ndim ? x_upper[d] : 1.0;
        w.per[d] = d < ndim ? (periodic ? periodic[d] != 0 : 1) : 0;
        if (d < ndim && !(w.hi[d] > w.lo[d])) return fail(IBTK_LE_ERR_ARG, "empty domain");
    }
    w.ndim = ndim;
    if (set_device(ctx)) return IBTK_LE_ERR_DEVICE;
    HIP_TRY(launch_wrap_positions(w, n, X_dev, ctx->stream));
    return IBTK_LE_OK;
}

// endDataRedistribution's reorder of an LData (LDataManager.cpp:1823-1917): node i of
// the new numbering takes the old row order_dev[i] (depth doubles per node).
extern "C" int ibtk_le_ldata_reorder(ibtk_le_ctx ctx, const int* order_dev, int n, const double* in_dev, int depth,
                                     double* out_dev) {
    if (!ctx) return fail(IBTK_LE_ERR_ARG, "null context");
    if (n < 0 || depth < 1) return fail(IBTK_LE_ERR_ARG, "bad sizes");
    if (n == 0) return IBTK_LE_OK;
    if (!order_dev || !in_dev || !out_dev) return fail(IBTK_LE_ERR_ARG, "null array");
    if (in_dev == out_dev) return fail(IBTK_LE_ERR_ARG, "reorder needs distinct input and output");
    if (set_device(ctx)) return IBTK_LE_ERR_DEVICE;
    HIP_TRY(launch_rows_gather(order_dev, n, in_dev, depth, out_dev, ctx->stream));
    return IBTK_LE_OK;
}

// LDataManager::computeNodeDistribution's local numbering (LDataManager.cpp:
// 2839-3027) for one patch: order_dev[i] = the input index of the marker that
// gets local index i; markers in cells of the patch box first, in box order (x
// fastest) and input order within a cell, then the markers outside the box in
// input order.  *n_interior (host, may be null) = the count inside the box.
extern "C" int ibtk_le_local_numbering(ibtk_le_ctx ctx, const ibtk_le_patch_geom* geom, const double* X_dev,
                                       int n_markers, int* order_dev, int* n_interior) {
    if (!ctx) return fail(IBTK_LE_ERR_ARG, "null context");
    if (int rc = check_geom(geom)) return rc;
    if (n_markers < 0) return fail(IBTK_LE_ERR_ARG, "negative size");
    if (n_markers > 0 && (!X_dev || !order_dev)) return fail(IBTK_LE_ERR_ARG, "null array");
    if (n_interior) *n_interior = 0;
    if (n_markers == 0) return IBTK_LE_OK;
    unsigned long long ncells = 1;
    for (int k = 0; k < geom->ndim; ++k) ncells *= (unsigned long long)(geom->iupper[k] - geom->ilower[k] + 1);
    if (ncells >= 0xffffffffull) return fail(IBTK_LE_ERR_RANGE, "patch box has %llu cells", ncells);
    if (set_device(ctx)) return IBTK_LE_ERR_DEVICE;
    ImageDesc d;
    std::memset(&d, 0, sizeof(d));
    d.ndim = geom->ndim;
    for (int k = 0; k < geom->ndim; ++k) {
        d.xlo[k] = geom->x_lower[k];
        d.xup[k] = geom->x_upper[k];
        d.dx[k] = geom->dx[k];
        d.ilo[k] = geom->ilower[k];
        d.ihi[k] = geom->iupper[k];
    }
    int rc;
    const size_t n = (size_t)n_markers;
    if ((rc = ctx->keys_in.ensure(2 * sizeof(unsigned) * n))) return rc;  // keys in | keys out
    if ((rc = ctx->vals_in.ensure(sizeof(int) * n))) return rc;
    if ((rc = ctx->counts.ensure(sizeof(int)))) return rc;
    const hipStream_t s = ctx->stream;
    unsigned* kin = ctx->keys_in.as<unsigned>();
    unsigned* kout = kin + n;
    HIP_TRY(hipMemsetAsync(ctx->counts.p, 0, sizeof(int), s));
    HIP_TRY(launch_cell_keys(d, X_dev, n_markers, (unsigned)ncells, kin, ctx->vals_in.as<int>(), ctx->counts.as<int>(),
                             s));
    int end_bit = 1;
    while ((1ull << end_bit) <= ncells) ++end_bit;
    size_t tb = 0;
    HIP_TRY(launch_sort(nullptr, tb, kin, kout, ctx->vals_in.as<int>(), order_dev, n_markers, end_bit, s));
    if ((rc = ctx->temp.ensure(tb))) return rc;
    tb = ctx->temp.cap;
    HIP_TRY(launch_sort(ctx->temp.p, tb, kin, kout, ctx->vals_in.as<int>(), order_dev, n_markers, end_bit, s));
    if (n_interior) {
        HIP_TRY(hipMemcpyAsync(n_interior, ctx->counts.p, sizeof(int), hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
    }
    return IBTK_LE_OK;
}

extern "C" int ibtk_le_mark_stencils(ibtk_le_ctx ctx, ibtk_le_markers m, int kernel, int centering, int axis,
                                     const ibtk_le_patch_geom* geom, unsigned char* const* masks_dev, int q_depth,
                                     const double* X_dev) {
    Params p;
    if (int rc = prepare(ctx, m, kernel, geom, X_dev, p)) return rc;
    const int nc = ncomponents(geom, centering, q_depth, centering == IBTK_LE_SIDE || centering == IBTK_LE_EDGE
                                                            ? geom->ndim
                                                            : q_depth);
    if (nc < 0) return -nc;
    if (nc > MAXC) return fail(IBTK_LE_ERR_ARG, "mark_stencils: at most %d components", MAXC);
    if (m->n == 0) return IBTK_LE_OK;
    if (set_device(ctx)) return IBTK_LE_ERR_DEVICE;
    std::vector<double*> dummy(nc, reinterpret_cast<double*>(16));
    ibtk_le_patch_geom gp = *geom;  // the masks are packed whatever the arrays' pitch
    gp.pitch[0] = gp.pitch[1] = 0;
    if (int rc = make_comps(&gp, centering, axis, dummy.data(), q_depth, q_depth, 0, nc, p)) return rc;
    unsigned char* mk[4] = {nullptr, nullptr, nullptr, nullptr};
    for (int c = 0; c < nc; ++c) {
        if (!masks_dev[c]) return fail(IBTK_LE_ERR_ARG, "null mask");
        mk[c] = masks_dev[c];
    }
    HIP_TRY(launch_mark(geom->ndim, kernel, p, m->n, mk, ctx->stream));
    return IBTK_LE_OK;
}
