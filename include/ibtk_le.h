/*
 * ibtk_le.h -- C-ABI of the MI355X-native Lagrangian-Eulerian coupling path.
 *
 * This library replaces the Fortran kernels behind IBTK::LEInteractor
 * (ibtk/src/lagrangian/LEInteractor.cpp, ibtk/src/lagrangian/fortran/
 * lagrangian_interaction{2,3}d.f.m4) with hand-written CDNA4 (gfx950) HIP
 * kernels.  Three levels are exported:
 *
 *  1. Device-resident API (ibtk_le_*): every array pointer is a device pointer;
 *     work is stream-ordered on the context's HIP stream; nothing blocks unless
 *     the function says so.  This is the level bench.py measures.
 *  2. Fortran-symbol host shims (lagrangian_<kernel>_{interp,spread}{2,3}d_):
 *     the exact symbols and by-reference signatures LEInteractor.cpp:68-619
 *     declares (IBTK_FC_FUNC_ lowercase + trailing underscore), host memory in
 *     and out (H2D -> kernel -> D2H).  Drop-in for the Fortran objects.
 *  3. A C++ LEInteractor facade (include/ibtk_le/LEInteractor.h) over light
 *     patch/data views, mirroring ibtk/include/ibtk/LEInteractor.h:100-993.
 *
 * Error convention (replaces TBOX_ERROR aborts, LEInteractor.cpp:679,2421,2740):
 * every function returns an ibtk_le_status; ibtk_le_last_error() describes the
 * most recent failure of the calling thread.
 */
#ifndef IBTK_LE_H
#define IBTK_LE_H

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes -------------------------------------------------------- */
typedef enum {
    IBTK_LE_OK = 0,
    IBTK_LE_ERR_UNKNOWN_KERNEL = 1, /* LEInteractor.cpp:679 "Unknown kernel function"        */
    IBTK_LE_ERR_GHOST_WIDTH = 2,    /* LEInteractor.cpp:2421, 2740 "insufficient ghost cells" */
    IBTK_LE_ERR_DEPTH = 3,          /* LEInteractor.cpp:769, 1627 side/edge depth mismatch   */
    IBTK_LE_ERR_ARG = 4,            /* invalid argument (null pointer, bad dim, bad box)     */
    IBTK_LE_ERR_DEVICE = 5,         /* HIP runtime error                                     */
    IBTK_LE_ERR_NOMEM = 6,          /* device allocation failed                              */
    IBTK_LE_ERR_RANGE = 7,          /* index space too large for the 32-bit bin keys         */
    IBTK_LE_ERR_INVARIANT = 8       /* a device-side consistency check failed                */
} ibtk_le_status;

/* ---- kernel functions (LEInteractor::getStencilSize, LEInteractor.cpp:668-682) */
typedef enum {
    IBTK_LE_KERNEL_PIECEWISE_CONSTANT = 0,
    IBTK_LE_KERNEL_DISCONTINUOUS_LINEAR = 1,
    IBTK_LE_KERNEL_PIECEWISE_LINEAR = 2,
    IBTK_LE_KERNEL_PIECEWISE_CUBIC = 3,
    IBTK_LE_KERNEL_IB_3 = 4,
    IBTK_LE_KERNEL_IB_4 = 5,
    IBTK_LE_KERNEL_IB_4_W8 = 6,
    IBTK_LE_KERNEL_IB_6 = 7,
    IBTK_LE_KERNEL_BSPLINE_4 = 8, /* not in the reference: cubic B-spline */
    IBTK_LE_KERNEL_USER_DEFINED = 9 /* LEInteractor::s_kernel_fcn: ibtk_le_user_interp / ibtk_le_user_spread */
} ibtk_le_kernel;

/* ---- data centerings (SAMRAI pdat::{Cell,Side,Node,Edge}Data) ---------------- */
typedef enum {
    IBTK_LE_CELL = 0, /* one array, depth q_depth, unshifted frame                      */
    IBTK_LE_SIDE = 1, /* NDIM arrays (one per axis), depth 1, x_lower[axis] -= dx/2     */
    IBTK_LE_NODE = 2, /* one array, depth q_depth, x_lower -= dx/2 in every dim         */
    IBTK_LE_EDGE = 3  /* 3D only: NDIM arrays, every dim but `axis` shifted             */
} ibtk_le_centering;

/* Patch geometry: the cell box, the ghost width of the Eulerian data and the
 * Cartesian patch geometry (CartesianPatchGeometry::getDx/getXLower/getXUpper).
 *
 * pitch: the layout of the Eulerian arrays in device memory.  {0, 0} is SAMRAI's
 * ArrayData layout, every array packed to its own ghosted extent (n0, n1, n2).
 * Otherwise every array of the patch (each side axis, each depth) has row stride
 * pitch[0] >= n0 and plane stride pitch[0] * pitch[1] (pitch[1] >= n1; 0 = n1);
 * depth k of a cell/node array starts k * pitch[0] * pitch[1] * n2 elements in.
 * With pitch[0] a multiple of 16 and 128-byte aligned array pointers, every
 * 32-point column row the 3-D sweeps stream is two whole 128-byte lines (the
 * sweeps' columns start at ilower - gcw + a multiple of 16 in x).  3-D single-
 * patch calls honour it; the level calls, the 2-D calls, ibtk_le_mark_stencils'
 * masks and the host Fortran shims take packed arrays only (pitch {0, 0}). */
typedef struct {
    int ndim;          /* 2 or 3 */
    int ilower[3];     /* patch box lower (cell indices) */
    int iupper[3];     /* patch box upper (inclusive)   */
    int gcw[3];        /* ghost cell width of the Eulerian arrays */
    double dx[3];
    double x_lower[3];
    double x_upper[3];
    int pitch[2];      /* array row / plane pitch in elements; {0, 0} = packed */
} ibtk_le_patch_geom;

typedef struct ibtk_le_ctx_s* ibtk_le_ctx;
typedef struct ibtk_le_markers_s* ibtk_le_markers;

/* ---- kernel-string helpers ---------------------------------------------------- */
/* Returns the kernel id for "IB_4", "IB_6", ... or -1 (LEInteractor.cpp:668-682). */
int ibtk_le_kernel_from_name(const char* name);

/* The USER_DEFINED kernel function: LEInteractor::s_kernel_fcn and
 * s_kernel_fcn_stencil_size (LEInteractor.h:100-101, LEInteractor.cpp:651-652), a
 * host function phi(r) of the signed distance in grid spacings, IB_4's
 * (ib4_kernel_fcn, LEInteractor.cpp:629-648) with stencil size 4 until set.
 * fcn == NULL restores the default.  Any stencil_size >= 1 (the spread's per-call
 * contribution count n * S^NDIM must stay below 2^31). */
typedef double (*ibtk_le_user_kernel_fn)(double r);
/* IB_4's kernel function, the reference's default s_kernel_fcn (ib4_kernel_fcn,
 * LEInteractor.cpp:629-651). */
double ibtk_le_ib4_kernel_fcn(double r);
int ibtk_le_set_user_kernel(ibtk_le_user_kernel_fn fcn, int stencil_size);
int ibtk_le_user_kernel(ibtk_le_user_kernel_fn* fcn, int* stencil_size);
const char* ibtk_le_kernel_name(int kernel);
/* LEInteractor::getStencilSize / getMinimumGhostWidth (LEInteractor.cpp:668-687). */
int ibtk_le_stencil_size(int kernel);
int ibtk_le_min_ghost_width(int kernel);
const char* ibtk_le_last_error(void);
const char* ibtk_le_version(void);

/* ---- context -------------------------------------------------------------------- */
/* `stream` is a hipStream_t (NULL = the default stream).  The context caches the
 * workspace the binning and sort steps need, so repeated calls allocate nothing. */
int ibtk_le_ctx_create(int device, void* stream, ibtk_le_ctx* out);
int ibtk_le_ctx_destroy(ibtk_le_ctx ctx);
int ibtk_le_ctx_set_stream(ibtk_le_ctx ctx, void* stream);
/* Restricts the next 3-D interp / spread calls on this context to a subset of
 * their work items (mode 1: the items whose planes -- interp: the planes it reads,
 * spread: the planes it owns -- all lie in [zlo, zhi], absolute z indices; mode 2:
 * the other items; mode 0: every item, the default).  A z-slab rank computes
 * its interior items while the halo exchange is in flight and the boundary
 * items after it; the two calls together equal one unrestricted call bit for
 * bit (each grid point is owned by exactly one item).  While zlo <= zhi, the
 * markers binned on this context (any mode) cut their sweep items at the
 * window's edges, so the boundary items are only the planes next to them.
 * 2-D calls ignore the window.  Replaces no reference entry point: the
 * reference overlaps nothing (RefineSchedule::fillData, LDataManager.cpp:748). */
int ibtk_le_ctx_set_plane_window(ibtk_le_ctx ctx, int mode, int zlo, int zhi);
/* Waits for the context stream and reports device-side invariant failures
 * latched by earlier calls (IBTK_LE_ERR_INVARIANT), then clears them: flag 1 / 2 a
 * stencil left its staged region / bin bounds, 4 an interior list entry missing from a
 * level's binned lists, 8 a fixed-capacity migration overflowed, 16 a 3-D spread's
 * candidate stream reached 2^31 entries (it holds up to 4 sorted positions a marker,
 * 16 bytes of device memory a marker, kept with the binning). */
int ibtk_le_ctx_synchronize(ibtk_le_ctx ctx);

/* ---- marker binning (device LIndexSetData / LDataManager re-binning) --------------
 * Replaces the per-patch index bookkeeping LEInteractor::buildLocalIndices
 * (LEInteractor.cpp:3031-3108) hands to the Fortran: it takes the list of
 * (local marker index, periodic shift) pairs -- `indices_dev`/`Xshift_dev`, or
 * NULL/NULL for the identity list 0..n-1 with zero shifts -- and sorts it on the
 * device by the stencil anchor cell of X(s)+Xshift (stable radix sort; 3-D:
 * buckets of (anchor plane, 32x16-cell column, reach band); 2-D: bricks of 16^2
 * cells).  The handle keeps device copies of the sorted list. */
int ibtk_le_markers_create(ibtk_le_ctx ctx, ibtk_le_markers* out);
int ibtk_le_markers_destroy(ibtk_le_markers m);
int ibtk_le_markers_bin(ibtk_le_ctx ctx, ibtk_le_markers m, const ibtk_le_patch_geom* geom, int kernel,
                        const double* X_dev, const int* indices_dev, const double* Xshift_dev, int nindices);
/* The same for a fixed-capacity marker array whose length lives on the device
 * (*n_dev <= capacity; a migration's output, no host sync): rows [n_dev, capacity)
 * are binned outside -- interp writes 0 to their Q rows, spread skips them -- so
 * Q/F arrays must hold capacity rows.  3-D, identity list. */
int ibtk_le_markers_bin_count(ibtk_le_ctx ctx, ibtk_le_markers m, const ibtk_le_patch_geom* geom, int kernel,
                              const double* X_dev, int capacity, const int* n_dev);
/* Re-bin the list of the last ibtk_le_markers_bin / _bin_count / ibtk_le_level_bin call
 * on `m` (same entries, shifts, patches and kernel) at new positions X_dev (the
 * markers moved, as between two steps of IBMethod's explicit loop).  The result --
 * sorted order, bucket starts, sorted positions, sweep items -- is exactly that of
 * binning again, but it is computed from the previous order: the entries whose
 * bucket did not change keep their relative order and the others are inserted
 * (with nothing moved, one pass over the list).  No host sync.  Replaces the
 * per-step re-binning of LDataManager's LIndexSetData (LDataManager.cpp:1446-1493,
 * IndexUtilities-inl.h:66-89) after a position update.  After ibtk_le_markers_bin_count
 * the re-binning reads the device count n_dev of that call again: it must stay valid
 * (and hold the list's length) until the next full binning of `m`. */
int ibtk_le_markers_rebin(ibtk_le_ctx ctx, ibtk_le_markers m, const double* X_dev);
/* Number of list entries, and device pointers to the sorted list (entry -> marker
 * index, and entry -> Xshift[NDIM]); valid until the next bin call. */
int ibtk_le_markers_count(ibtk_le_markers m);
/* Device pointer to the canonical order: order_dev[i] = position in the binned
 * list (0..count-1) of the i-th entry in canonical order.  Valid until the next
 * bin call; the caller may copy it to the host to feed the oracle the same list. */
int ibtk_le_markers_order(ibtk_le_markers m, const int** order_dev);

/* ---- interpolation / spreading on device-resident data --------------------------
 * q_dev[c] points at the ghosted Fortran-ordered array of component c:
 *   SIDE/EDGE: c = 0..NDIM-1, the array of axis c (SideData::getPointer(c)), depth 1
 *   CELL/NODE: c = 0 only, an array of depth q_depth (depth slowest)
 * Q_dev is the marker array in LData layout: AoS, Q_depth values per marker
 * (SIDE/EDGE: Q_depth == NDIM).  X_dev: AoS NDIM positions per marker.
 * The marker list is the one last binned into `m` (same kernel and geometry).
 * A list may name a marker several times (LIndexSetData's ghost-box list holds
 * its periodic images): spread adds every entry; interp writes Q(:, s) from the
 * LAST entry naming s, as the Fortran's sequential l-loop overwrites it.
 *
 * interp:  Q(d, s) = sum_i w_i(X(s)+Xshift) q(i, d)   for every listed s
 *          (LEInteractor.cpp:970-1055 / lagrangian_<k>_interp3d, f.m4:1258-1385)
 * spread:  q(i, d) += sum_s w_i(X(s)+Xshift) Q(d, s) / (dx0 dx1 [dx2])
 *          summed per grid point in a fixed order (work-item-private LDS
 *          accumulation, no global atomics): deterministic and bit-stable run
 *          to run
 *          (LEInteractor.cpp:1828-1913 / lagrangian_<k>_spread3d, f.m4:1395-1522) */
int ibtk_le_interp(ibtk_le_ctx ctx, ibtk_le_markers m, int kernel, int centering, int axis,
                   const ibtk_le_patch_geom* geom, const double* const* q_dev, int q_depth, double* Q_dev,
                   int Q_depth, const double* X_dev);
int ibtk_le_spread(ibtk_le_ctx ctx, ibtk_le_markers m, int kernel, int centering, int axis,
                   const ibtk_le_patch_geom* geom, double* const* q_dev, int q_depth, const double* Q_dev,
                   int Q_depth, const double* X_dev);

/* USER_DEFINED interpolation and spreading: LEInteractor::userDefinedInterpolate /
 * userDefinedSpread (LEInteractor.cpp:3141-3266, 3268-3393), the branches of the
 * private interpolate()/spread() at :2688 and :3007.  Arguments as ibtk_le_interp /
 * ibtk_le_spread, with the list given directly (no binning): indices_dev (n list
 * entries -> marker, NULL: entry l is marker l) and Xshift_dev (n x NDIM, NULL:
 * zero).  Per entry and dimension: stencil centre floor((X+Xshift-x_lower)/dx) +
 * ilower; an even stencil starts below or above it as the UNSHIFTED X lies below
 * or above the cell centre (:3188, as the reference compares); the stencil is
 * clipped into the ghost box; weights phi((X+Xshift - x_i)/dx).  phi is a host
 * function: the host evaluates it (one synchronization per call), the device
 * sums.  interp: Q(d, s) = sum w0 w1 [w2] q in the reference's loop order (the
 * last entry naming s writes it); spread: q += w0 w1 [w2] Q(d, s) / (dx0 dx1
 * [dx2]), every grid point summed in list order (bit-stable; the reference's
 * sequential order). */
int ibtk_le_user_interp(ibtk_le_ctx ctx, int centering, int axis, const ibtk_le_patch_geom* geom,
                        const double* const* q_dev, int q_depth, double* Q_dev, int Q_depth, const double* X_dev,
                        const int* indices_dev, const double* Xshift_dev, int n);
int ibtk_le_user_spread(ibtk_le_ctx ctx, int centering, int axis, const ibtk_le_patch_geom* geom,
                        double* const* q_dev, int q_depth, const double* Q_dev, int Q_depth, const double* X_dev,
                        const int* indices_dev, const double* Xshift_dev, int n);

/* Density-weighted spread, f += S (F ds): LDataManager::spread with ds_data
 * (LDataManager.cpp:398-470), which forms F_ds[k][d] = F[k][d] * ds[k] and then
 * spreads it.  ds_dev holds one double per marker (indexed like Q_dev's markers).
 * The product is formed in the gather that stages F for the spread kernel, so it
 * costs no extra pass; the values spread are the rounded products, as in the
 * reference. */
int ibtk_le_spread_ds(ibtk_le_ctx ctx, ibtk_le_markers m, int kernel, int centering, int axis,
                      const ibtk_le_patch_geom* geom, double* const* q_dev, int q_depth, const double* Q_dev,
                      int Q_depth, const double* ds_dev, const double* X_dev);

/* ---- a level of patches (3-D) ------------------------------------------------------
 * LDataManager::spread / interp loop over the patches of a level, one LEInteractor
 * call per patch (LDataManager.cpp:625-660, 763-807).  Here one launch per sweep
 * covers every patch: the patches' lists are binned together (bucket ranges per
 * patch, one device sort) and the sweep items of all patches form one table.
 * geoms[q]: patch q's box, ghost width and geometry (one dx for the level);
 * entry_offsets (host, npatch + 1): patch q's list is entries [off[q], off[q+1])
 * of indices_dev / Xshift_dev (NULL/NULL: entry l is marker l, no shift) -- the
 * interior list for interp, the ghost-box list for spread, as LDataManager uses.
 * q_dev: the arrays of patch 0, then patch 1, ... (NDIM per patch for SIDE/EDGE,
 * one for CELL/NODE).  Results equal the per-patch calls' (interp bit for bit;
 * spread in each patch's own fixed order). */
int ibtk_le_level_bin(ibtk_le_ctx ctx, ibtk_le_markers m, int npatch, const ibtk_le_patch_geom* geoms, int kernel,
                      const double* X_dev, const int* entry_offsets, const int* indices_dev,
                      const double* Xshift_dev);
int ibtk_le_level_interp(ibtk_le_ctx ctx, ibtk_le_markers m, int kernel, int centering, int axis,
                         const double* const* q_dev, int q_depth, double* Q_dev, int Q_depth, const double* X_dev);
int ibtk_le_level_spread(ibtk_le_ctx ctx, ibtk_le_markers m, int kernel, int centering, int axis,
                         double* const* q_dev, int q_depth, const double* Q_dev, int Q_depth, const double* X_dev);
/* q := 0 on every patch array (ghosts included), then ibtk_le_level_spread, in one
 * launch: LDataManager::spread's setToScalar(f, 0, interior_only = false) fused with
 * its patch loop (LDataManager.cpp:588-654).  The sweep's items start their owned
 * points from 0 instead of reading them; items no marker reaches store zeros.
 * Bitwise ibtk_le_level_zero followed by ibtk_le_level_spread. */
int ibtk_le_level_zero_spread(ibtk_le_ctx ctx, ibtk_le_markers m, int kernel, int centering, int axis,
                              double* const* q_dev, int q_depth, const double* Q_dev, int Q_depth,
                              const double* X_dev);
/* One binning for both sweeps: m binned on the ghost-box lists (the spread's), then
 * told the interior lists (interior_offsets on the host, npatch + 1; indices on the
 * device; markers 0 .. n_markers-1): later level interps on m write Q only from the
 * entries the interior lists name (each patch's interior list is the unshifted
 * sub-list of its ghost-box list whose cells lie in the patch box, LIndexSetData.cpp:
 * 111-166), so results equal interp over a binning of the interior lists bit for bit.
 * Cleared by the next bin.  An interior entry missing from its patch's binned list
 * raises device flag 4 (ibtk_le_ctx_synchronize).  After ibtk_le_markers_rebin, a call
 * with the same offsets, index pointer and n_markers as the last one since the last
 * full binning is a no-op on the device when no marker changed bucket (the lists are
 * taken to be unchanged between binnings, as the re-binning takes the binned ones). */
int ibtk_le_level_select_interior(ibtk_le_ctx ctx, ibtk_le_markers m, int n_markers, const int* interior_offsets,
                                  const int* interior_indices_dev);
/* Forget the selection kept by ibtk_le_level_select_interior: the next call recomputes it
 * whatever its arguments (a caller that rewrites the interior lists in place, or frees them
 * and allocates new ones, calls this first). */
int ibtk_le_level_select_interior_reset(ibtk_le_markers m);
/* Zeroes every patch array of a level, ghosts included, in one launch: the
 * f := 0 before LDataManager::spread accumulates into the level (its
 * f_data_ops->setToScalar(f_data_idx, 0.0, interior_only = false),
 * LDataManager.cpp:596).  q_dev as
 * ibtk_le_level_fill_ghosts (NDIM arrays per patch for SIDE / EDGE; one array of
 * depth q_depth for CELL / NODE), each contiguous. */
int ibtk_le_level_zero(ibtk_le_ctx ctx, int npatch, const ibtk_le_patch_geom* geoms, int centering,
                       double* const* q_dev, int q_depth);
/* Ghost fill of a level of equal patches tiling a box, periodic in the dims
 * periodic[d] != 0 (NULL: all): every ghost point of every patch array takes the
 * value of the patch owning its (wrapped) index -- the RefineSchedule::fillData
 * LDataManager::interp runs before interpolating (LDataManager.cpp:748-751).
 * SIDE (NDIM arrays per patch; the face shared by two patches is the upper
 * patch's) or CELL (one array of depth q_depth per patch). */
int ibtk_le_level_fill_ghosts(ibtk_le_ctx ctx, int npatch, const ibtk_le_patch_geom* geoms, int centering,
                              double* const* q_dev, int q_depth, const int* periodic);
/* ibtk_le_level_fill_ghosts(m's patches, periodic) followed by ibtk_le_level_interp,
 * Q bit for bit, in one sweep: a patch's ghost point is read in the neighbour patch the
 * fill would copy it from (the patch owning its wrapped index, at the same global
 * index), so no ghost value is written (across a non-periodic face, where the fill
 * copies nothing, the patch's own ghost values are read).  Fused when, per component, every patch's array lies within one 2-GB
 * address window (one allocation per component for the level, e.g.), the patches have
 * at least 32 + W - 1 cells in x and 16 + W - 1 in y (W: the kernel's stencil width),
 * and the data are SIDE or CELL of depth 1; otherwise the two calls. */
int ibtk_le_level_fill_interp(ibtk_le_ctx ctx, ibtk_le_markers m, int kernel, int centering, int axis,
                              double* const* q_dev, int q_depth, double* Q_dev, int Q_depth, const double* X_dev,
                              const int* periodic);

/* ---- helpers for a single periodic patch (uniform finest level) -----------------
 * Fill the ghost layers of the arrays of `centering` from the periodic interior
 * (the RefineSchedule::fillData the caller runs before interp, LDataManager.cpp:750). */
int ibtk_le_fill_periodic_ghosts(ibtk_le_ctx ctx, const ibtk_le_patch_geom* geom, int centering,
                                 double* const* q_dev, int q_depth, const int* periodic);
/* ibtk_le_fill_periodic_ghosts followed by ibtk_le_interp, with the same Q bit for bit,
 * in one sweep for a 3-D column binning: the interp reads every ghost point of the
 * ghost box at its periodic image in the periodic dims (the value the fill copies
 * there) and writes no ghost value (q is not modified).  periodic NULL: every dim.
 * Other binnings: the two calls. */
int ibtk_le_fill_interp(ibtk_le_ctx ctx, ibtk_le_markers m, int kernel, int centering, int axis,
                        const ibtk_le_patch_geom* geom, const double* const* q_dev, int q_depth, double* Q_dev,
                        int Q_depth, const double* X_dev, const int* periodic);
/* Spreading in ghost-region-sum mode: zero the ghost layers before spreading the
 * interior markers, then fold every ghost value back onto its periodic interior
 * image (dims folded slowest first, one source per destination per pass:
 * deterministic).  The multi-GPU path uses the same fold along x/y and an RCCL
 * exchange along z. */
int ibtk_le_zero_ghosts(ibtk_le_ctx ctx, const ibtk_le_patch_geom* geom, int centering, double* const* q_dev,
                        int q_depth);
/* ibtk_le_zero_ghosts followed by ibtk_le_spread, bit for bit, in one sweep for a 3-D
 * column binning: the spread's items start their owned ghost points (outside the data
 * box) from 0 instead of reading them, and items no marker reaches store the zeros
 * (the ghost zeroing of LDataManager::spread, LDataManager.cpp:587-671, with no
 * separate pass over the ghost layers).  Other binnings: the two calls. */
int ibtk_le_zero_ghosts_spread(ibtk_le_ctx ctx, ibtk_le_markers m, int kernel, int centering, int axis,
                               const ibtk_le_patch_geom* geom, double* const* q_dev, int q_depth,
                               const double* Q_dev, int Q_depth, const double* X_dev);
/* The target as LDataManager::spread hands it to LEInteractor::spread: every point of
 * q set to 0, ghosts included (LDataManager.cpp:596, setToScalar(f, 0,
 * interior_only = false)), then ibtk_le_spread into it -- bit for bit those two steps.
 * A 3-D column binning does both in the spread's sweep (items start every owned point
 * from 0 and never read q; items no marker reaches store zeros), so q is written once
 * and not read.  Other binnings (2-D, an empty list): the zeroing (pitched arrays: the
 * whole span, row padding included), then ibtk_le_spread. */
int ibtk_le_zero_spread(ibtk_le_ctx ctx, ibtk_le_markers m, int kernel, int centering, int axis,
                        const ibtk_le_patch_geom* geom, double* const* q_dev, int q_depth, const double* Q_dev,
                        int Q_depth, const double* X_dev);
int ibtk_le_fold_periodic_ghosts(ibtk_le_ctx ctx, const ibtk_le_patch_geom* geom, int centering,
                                 double* const* q_dev, int q_depth, const int* periodic);
/* Physical-boundary ghost operators for side-centred data on one patch
 * (CartSideRobinPhysBdryOp, CartSideRobinPhysBdryOp.cpp:358-493, arithmetic of
 * cartphysbdryop{2,3}d.f.m4).  adjoint = 0: setPhysicalBoundaryConditions, the
 * ghost fill before interpolation; adjoint = 1: accumulateFromPhysicalBoundary
 * Data, the fold LDataManager::spread runs after spreading (LDataManager.cpp:
 * 655-659).  u_dev[axis]: the ghosted side arrays; the ghost width must be the
 * same in every dim (the reference asserts it, :519-527).  physical[2 d + upper]
 * flags a face on a non-periodic physical boundary (edges/corners are boxes
 * whose faces are all physical); acoef/bcoef/gcoef[c * 2 ndim + loc] are the
 * Robin coefficients of component c on face loc, constant over the face
 * (RobinBcCoefStrategy::setBcCoefs, index NDIM*depth + axis with depth 0).
 * Periodic dims are folded/filled separately (ibtk_le_{fold,fill}_periodic_
 * ghosts), before the physical fold and after the physical fill.  Bitwise equal
 * to the serial Fortran order. */
int ibtk_le_phys_bdry_side(ibtk_le_ctx ctx, const ibtk_le_patch_geom* geom, double* const* u_dev,
                           const int* physical, const double* acoef, const double* bcoef, const double* gcoef,
                           int adjoint);
/* Local numbering of one patch's markers (LDataManager::computeNodeDistribution,
 * LDataManager.cpp:2839-3027, cells by IndexUtilities::getCellIndex): order_dev[i]
 * is the input index of the marker given local index i.  Markers whose cell is in
 * the patch box come first, in box iteration order (x fastest), input order within
 * a cell (a stable device radix sort); the others follow in input order.  If
 * n_interior is not NULL it receives the count inside the box (this synchronises
 * the stream). */
int ibtk_le_local_numbering(ibtk_le_ctx ctx, const ibtk_le_patch_geom* geom, const double* X_dev, int n_markers,
                            int* order_dev, int* n_interior);
/* Build the list of interior markers and of their periodic images that fall in the
 * ghost box (LIndexSetData::cacheLocalIndices, LIndexSetData.cpp:83-169, for one
 * patch covering a periodic domain; getCellIndex, IndexUtilities-inl.h:66-89).
 * Order: the reference's -- the ghost box's cells in iteration order (x fastest;
 * an image sits in its shifted cell), each cell's markers by index.  Writes up to
 * `capacity` entries into indices_dev / Xshift_dev (NDIM per entry) and the
 * entry count into *count (host).  ghost = 0 gives the interior list.
 * If the list needs more than `capacity` entries, nothing is written, *count
 * holds the required size and IBTK_LE_ERR_ARG is returned.  Synchronises. */
int ibtk_le_periodic_index_list(ibtk_le_ctx ctx, const ibtk_le_patch_geom* geom, const double* X_dev,
                                int n_markers, int ghost, const int* periodic, int* indices_dev,
                                double* Xshift_dev, int capacity, int* count);
/* The same lists with the Lagrangian index of every marker (lag_dev[s]; NULL = s):
 * within a cell the entries follow the LNodeSet order, sorted by Lagrangian index
 * and uniqued (LDataManager.cpp:1487-1493: of markers sharing a cell and a Lagrangian
 * index the lowest marker index is kept; the reference leaves which one unspecified).
 * With lag_dev the entry count is known only after uniquing: a capacity below it
 * writes nothing and returns IBTK_LE_ERR_ARG with *count = the required size.
 * which = 0: every entry (d_local_petsc_indices /
 * d_periodic_shifts), 1: the cells of the patch box (d_interior_*), 2: the other
 * ghost-box cells (d_ghost_*) -- the three lists cacheLocalIndices caches.
 * SAMRAI's IndexData walks its items in insertion order; the lists take the
 * box iteration order, which that insertion order follows for sets appended
 * cell by cell (LDataManager.cpp:1446-1482 walks the cells in box order). */
int ibtk_le_index_set_list(ibtk_le_ctx ctx, const ibtk_le_patch_geom* geom, const double* X_dev, const int* lag_dev,
                           int n_markers, int ghost, const int* periodic, int which, int* indices_dev,
                           double* Xshift_dev, int capacity, int* count);
/* LEInteractor::buildLocalIndices for a box that is neither the patch box nor the
 * ghost box (LEInteractor.cpp:3070-3106): the entries of the which = 0 list above
 * whose cell -- the cell of the index set's item, an image's shifted cell -- lies in
 * [box_lo, box_hi], in the same order and with the same periodic shifts (the
 * reference's per-cell offsets, -/+ periodic_shift * dx beyond the patch's periodic
 * sides, are the images' shifts).  box == the patch box gives the which = 1 list,
 * box == the ghost box the which = 0 list.  cells_dev (NULL: not written) receives
 * NDIM ints per entry: its cell.  Count and capacity as above; synchronises. */
int ibtk_le_index_set_box_list(ibtk_le_ctx ctx, const ibtk_le_patch_geom* geom, const double* X_dev,
                               const int* lag_dev, int n_markers, int ghost, const int* periodic, const int* box_lo,
                               const int* box_hi, int* indices_dev, double* Xshift_dev, int* cells_dev, int capacity,
                               int* count);
/* The entries of a cached list whose cell (cells_dev, NDIM ints per entry, as
 * ibtk_le_index_set_box_list writes them) lies in [box_lo, box_hi], order kept:
 * buildLocalIndices' box branch over a cached index set.  Xshift_dev may be NULL
 * (then Xshift_out is not written).  Synchronises. */
int ibtk_le_list_in_box(ibtk_le_ctx ctx, int ndim, const int* cells_dev, const int* indices_dev,
                        const double* Xshift_dev, int n, const int* box_lo, const int* box_hi, int* indices_out,
                        double* Xshift_out, int capacity, int* count);
/* LDataManager::computeNodeDistribution (LDataManager.cpp:2839-3027) for one patch
 * whose marker index data has `ghost` ghost cells: order_dev[i] = the input index
 * of the marker numbered i.  The local nodes (getCellIndex cell in the patch box)
 * come first, cell by cell in box order (x fastest), each cell by Lagrangian index
 * (lag_dev; NULL = input index) with repeated (cell, Lagrangian index) pairs kept
 * once (LDataManager.cpp:1487-1493); then the nonlocal nodes of the ghost cells in
 * ghost-box order.  Markers outside the ghost box are dropped.  *n_local and
 * *n_nonlocal (host) receive the counts.  Synchronises. */
int ibtk_le_node_distribution(ibtk_le_ctx ctx, const ibtk_le_patch_geom* geom, const double* X_dev,
                              const int* lag_dev, int n_markers, int ghost, int* order_dev, int* n_local,
                              int* n_nonlocal);

/* LDataManager::computeNodeDistribution (LDataManager.cpp:2874-2947) over the local
 * patches of one level, geoms[q] in PatchLevel order: equal patch boxes aligned to one
 * tiling of the domain [dom_lo, dom_hi] (periodic in the dims periodic[d] != 0; NULL =
 * all), cells by getCellIndex in the domain frame.  X_dev holds the rank's markers (its
 * own and the ghost nodes it holds), lag_dev their Lagrangian indices (NULL = the
 * marker index).  order_dev[i] = the input index of the marker that is node i:
 *   nodes 0 .. n_local-1: the markers in a local patch's box, patch by patch, the box's
 *     cells in box order (x fastest), a cell's set by Lagrangian index and uniqued
 *     (LDataManager.cpp:1487-1493, lowest marker index kept);
 *   then n_nonlocal nodes: the markers in some patch's ghost cells (periodic images
 *     included) whose Lagrangian index no local node has, one per index, at its first
 *     sighting -- patches in order, a patch's ghost box walked in box order, skipping
 *     its patch box (SAMRAI's BoxList::removeIntersections order is not vendored: that
 *     order is the box order here, parity unpinned).
 * Markers in no patch's ghost box are not numbered.  The global PETSc index of local
 * node i is node_offset + i, node_offset = the local counts of the lower ranks
 * (computeNodeOffsets, LDataManager.cpp:3029-3047: an all-gather the caller runs).
 * Synchronises. */
int ibtk_le_level_node_distribution(ibtk_le_ctx ctx, int npatch, const ibtk_le_patch_geom* geoms, const int* dom_lo,
                                    const int* dom_hi, const int* periodic, const double* X_dev, const int* lag_dev,
                                    int n_markers, int ghost, int* order_dev, int* n_local, int* n_nonlocal);
/* LIndexSetData::cacheLocalIndices (LIndexSetData.cpp:83-169) for every local patch of a
 * level in one call: the lists LDataManager::spread / interp hand LEInteractor per patch
 * (LDataManager.cpp:634-654, 763-807).  The patches as for ibtk_le_level_node_distribution
 * (equal boxes on one tiling of [dom_lo, dom_hi], periodic[d] != 0 periodic, NULL = all);
 * cells by getCellIndex in the domain frame, without Lagrangian indices (every marker is its
 * own node).
 *   interior lists: the markers whose cell lies in patch q's box, at interior_dev
 *     [interior_off[q], interior_off[q + 1]);
 *   ghost-box lists: the markers and their periodic images whose cell lies in patch q's
 *     box grown by `ghost`, at ghost_dev / Xshift_dev (NDIM doubles an entry: the image's
 *     shift, +-(dom_hi - dom_lo + 1) dx per periodic dim) [ghost_off[q], ghost_off[q + 1]).
 * Within a patch the entries follow (order 0) its (ghost) box's cells in box order, x
 * fastest, a cell's markers by index -- ibtk_le_periodic_index_list's order for one patch,
 * the reference's IndexData order -- or (order 1) the markers' order, a marker's images in
 * image order (the same sets; a sort by patch alone, fewer radix passes).
 * interior_off / ghost_off are host arrays of npatch + 1.  If a list needs more than its
 * capacity, both offset arrays are still written (off[npatch] = the size needed), that list
 * is not, and IBTK_LE_ERR_ARG is returned.  Synchronises. */
int ibtk_le_level_index_lists(ibtk_le_ctx ctx, int npatch, const ibtk_le_patch_geom* geoms, const int* dom_lo,
                              const int* dom_hi, const int* periodic, const double* X_dev, int n_markers, int ghost,
                              int order, int* interior_dev, int interior_cap, int* interior_off, int* ghost_dev,
                              double* Xshift_dev, int ghost_cap, int* ghost_off);
/* beginDataRedistribution's wrap of marker positions into the periodic domain
 * (LDataManager.cpp:1385-1399), in place on n (ndim)-records: per periodic dim
 * (periodic NULL: all) add / subtract the domain length while outside
 * [x_lower, x_upper), then clamp every dim into [x_lower, x_upper - DBL_EPSILON]. */
int ibtk_le_wrap_positions(ibtk_le_ctx ctx, int ndim, long long n, double* X_dev, const double* x_lower,
                           const double* x_upper, const int* periodic);
/* endDataRedistribution's reorder of an LData into the new numbering (the VecScatter of
 * LDataManager.cpp:1823-1917): out[i][k] = in[order_dev[i]][k], depth doubles per
 * node, device arrays, in and out distinct. */
int ibtk_le_ldata_reorder(ibtk_le_ctx ctx, const int* order_dev, int n, const double* in_dev, int depth,
                          double* out_dev);

/* Markers whose cell (IndexUtilities::getCellIndex against the patch box) lies in
 * [box_lo, box_hi], no periodic shifts: the list LEInteractor's X-only overloads
 * build (LEInteractor.cpp:3110-3139).  Marker-major order. */
int ibtk_le_box_index_list(ibtk_le_ctx ctx, const ibtk_le_patch_geom* geom, const double* X_dev, int n_markers,
                           const int* box_lo, const int* box_hi, int* indices_dev, int capacity, int* count);

/* Marker position update, elementwise over the n = M * NDIM doubles of the
 * device arrays (any layout, as long as all four share it):
 *   IBTK_LE_EULER, IBTK_LE_MIDPOINT:  X_new = dt * U0 + X_cur
 *     (IBMethod::eulerStep / midpointStep, IBMethod.cpp:619-655: VecWAXPY with U0 =
 *     U(current) or U(current + dt/2));
 *   IBTK_LE_TRAPEZOIDAL:  X_new = (dt/2 * U0 + X_cur) + dt/2 * U1
 *     (IBMethod::trapezoidalStep, IBMethod.cpp:657-681: VecWAXPY then VecAXPY, U0 =
 *     U(current), U1 = U(new)).
 * Each step is a rounded multiply and a rounded add, as PETSc's loops compute it.
 * X_new may alias X_cur.  U1 is ignored (may be NULL) unless TRAPEZOIDAL. */
enum { IBTK_LE_EULER = 0, IBTK_LE_MIDPOINT = 1, IBTK_LE_TRAPEZOIDAL = 2 };
int ibtk_le_position_update(ibtk_le_ctx ctx, int scheme, long long n, double dt, const double* X_cur_dev,
                            const double* U0_dev, const double* U1_dev, double* X_new_dev);

/* Position update fused with the z-slab migration classes (bench.py --move, ibamr_amd.slab.
 * migrate_device): X_new = the ibtk_le_position_update of (X_cur, U0, U1), wrapped
 * into [0, L) per dim as torch.remainder does; the markers' owners are the slabs of
 * their wrapped z cells (IndexUtilities::getCellIndex, LDataManager.cpp:1446; Nz
 * planes, nranks equal slabs).  order_dev (M ints) receives a stable partition of
 * the marker indices [staying | to rank-1 | to rank+1 | further], each part in
 * input order; counts_dev (4 ints, device) the part sizes.  Stream-ordered, no
 * host sync (the redistribution LDataManager.cpp:1504-1959 runs at regrid; SURVEY.md
 * 8(e) asks for it after every update).  X_new must not alias X_cur.  With two
 * ranks both neighbours are one rank: every leaver is in the second part. */
int ibtk_le_slab_update_partition(ibtk_le_ctx ctx, int scheme, long long M, double dt, const double* X_cur_dev,
                                  const double* U0_dev, const double* U1_dev, double* X_new_dev, const double* L,
                                  int Nz, int nranks, int rank, int* order_dev, int* counts_dev);
/* Fixed-capacity migration, no host sync (slab.update_and_migrate_fixed):
 * ibtk_le_slab_update_partition_count is the partition of the first *n_dev of
 * `capacity` rows; pack copies the down / up leavers of rows_dev ([capacity][depth]
 * doubles: X then the LData fields) into send buffers of send_cap rows each; after
 * the fixed-size exchange, unpack writes the stayers in order, then recv_counts[0]
 * rows of from_down and recv_counts[1] of from_up, into out_dev (out_cap rows) and
 * their number into *n_out_dev.  Leavers beyond send_cap, markers moving further
 * than one slab, or arrivals beyond out_cap raise device flag 8 (reported by
 * ibtk_le_ctx_synchronize): the caller sizes the buffers, the library never drops
 * a marker silently. */
int ibtk_le_slab_update_partition_count(ibtk_le_ctx ctx, int scheme, long long capacity, double dt,
                                        const double* X_cur_dev, const double* U0_dev, const double* U1_dev,
                                        double* X_new_dev, const double* L, int Nz, int nranks, int rank,
                                        const int* n_dev, int* order_dev, int* counts_dev);
int ibtk_le_slab_migrate_pack(ibtk_le_ctx ctx, const double* rows_dev, int depth, const int* order_dev,
                              const int* counts_dev, int send_cap, double* send_down_dev, double* send_up_dev);
int ibtk_le_slab_migrate_unpack(ibtk_le_ctx ctx, const double* rows_dev, int depth, const int* order_dev,
                                const int* counts_dev, const int* recv_counts_dev, const double* from_down_dev,
                                const double* from_up_dev, int send_cap, double* out_dev, int out_cap,
                                int* n_out_dev);

/* Diagnostics: masks_dev[c] (one byte per point of component c's ghosted array,
 * same layout) gets 1 at every point some listed stencil touches after clipping.
 * bench.py sums the masks for the exact algorithmic byte count |S_a|. */
int ibtk_le_mark_stencils(ibtk_le_ctx ctx, ibtk_le_markers m, int kernel, int centering, int axis,
                          const ibtk_le_patch_geom* geom, unsigned char* const* masks_dev, int q_depth,
                          const double* X_dev);

/* Diagnostics: number of device kernel launches issued by the last interp/spread/bin
 * call on this context, and the per-step timing of the last call's main kernel (ms,
 * measured with HIP events on the context stream when enabled). */
int ibtk_le_ctx_enable_timing(ibtk_le_ctx ctx, int enable);
/* Diagnostics: tuning overrides of the 3-D sweeps' work items (0 = default), both
 * taking effect at the next bin: "heavy" (own markers per item above which the
 * item is scheduled first; -1 never; default 4x the mean, at least 2048),
 * "seg_items" (target number of (column, segment)
 * items, which sets the segment length), "split_target" (own markers above
 * which a (column, segment) is cut into sub-segments), "min_piece" (planes per
 * sub-segment of a cut item, at least; default 8), "heavy_target" and
 * "heavy_min_piece" (the same for heavy items; defaults 2048 and 1), "strip" (column rows per
 * strip of the item order), "xcd_block" (light items over the XCDs in blocks of
 * this many table entries: 1 round-robin, -1 one range per XCD; default 8), and,
 * taking effect at the next interp, "interp3" (1: the three components of a one-patch
 * closed-form interp item in one workgroup -- each marker read once, each Q record written
 * whole; bitwise the same result; 0, the default: a workgroup per component), and,
 * taking effect at the next spread, "side_gather" (1: the 3-D spread's F gather on the
 * context's side stream, beside a candidate-stream rebuild; -1: in line before the sweep;
 * 0, the default: the side stream from 2^25 markers; bitwise the same result).
 * Interp results do not depend on them; spread results are bit-stable for fixed
 * settings and may differ in the last bits between settings (same-point adds
 * within one 64-candidate chunk follow its step and lane order, and the chunk
 * boundaries move with the items). */
int ibtk_le_ctx_tune(ibtk_le_ctx ctx, const char* key, int value);
double ibtk_le_ctx_last_kernel_ms(ibtk_le_ctx ctx);
/* Counted 3-D spread sweeps (a diagnostic for the LDS-atomic bound; one host sync
 * per launch): while enabled, each spread call records the ds_add_f64 it issues,
 * out[0] = wave-instructions, out[1] = lane adds (summed over its components). */
int ibtk_le_ctx_count_adds(ibtk_le_ctx ctx, int enable);
int ibtk_le_ctx_last_adds(ibtk_le_ctx ctx, unsigned long long* out);

#ifdef __cplusplus
}
#endif
#endif /* IBTK_LE_H */
