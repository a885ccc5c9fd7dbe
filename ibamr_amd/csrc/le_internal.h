// le_internal.h -- internal device-side descriptors of the LE coupling path.
// Not part of the C-ABI (include/ibtk_le.h is).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace ibtk_le {

// Kernel ids (== ibtk_le_kernel).
enum : int {
    K_PIECEWISE_CONSTANT = 0,
    K_DISCONTINUOUS_LINEAR = 1,
    K_PIECEWISE_LINEAR = 2,
    K_PIECEWISE_CUBIC = 3,
    K_IB_3 = 4,
    K_IB_4 = 5,
    K_IB_4_W8 = 6,
    K_IB_6 = 7,
    K_BSPLINE_4 = 8,
    K_COUNT = 9
};

// Host-visible copy of the kernel traits (le_stencil.h static_asserts agree):
// W = stencil points per dim; every stencil index of every centering frame lies
// in [key + LO, key + HI], key = the marker's cell-frame anchor.
struct KernelInfo {
    int W, LO, HI;
};
constexpr KernelInfo kKernelInfo[K_COUNT] = {
    {1, 0, 1},   // PIECEWISE_CONSTANT
    {2, -1, 2},  // DISCONTINUOUS_LINEAR
    {2, -1, 2},  // PIECEWISE_LINEAR
    {4, -2, 3},  // PIECEWISE_CUBIC
    {3, -1, 2},  // IB_3
    {4, -2, 2},  // IB_4
    {8, -4, 4},  // IB_4_W8
    {6, -3, 3},  // IB_6
    {4, -2, 2},  // BSPLINE_4
};

constexpr int MAXC = 4;        // components processed by one launch
constexpr int BRICK3 = 8;      // brick edge (cells) in 3-D: 8^3 = 512 cells
constexpr int BRICK2 = 16;     // brick edge in 2-D: 16^2 = 256 cells
constexpr int BLOCK = 256;     // threads per workgroup (4 waves)
constexpr int TILE = 4;        // bricks per tile edge

// One Eulerian array (a component of side data, or a depth slice of cell /
// node data) in SAMRAI's Fortran layout u(lo0:hi0, lo1:hi1, [lo2:hi2]).
struct CompDesc {
    double* u;       // device pointer to element (lo0, lo1, lo2)
    int lo[3];       // ghost box lower
    int hi[3];       // ghost box upper (inclusive)
    int ilower[3];   // the "ilower" argument the Fortran receives (data box lower)
    int iupper[3];   // the patch box upper: points past it (or below ilower) are the ghost
                     // points of the periodic ghost operations (a side array's face iupper+1 too)
    double xlo[3];   // the "x_lower" argument the Fortran receives (frame shift applied)
    int qcomp;       // which AoS component of Q this array pairs with
    int axis;        // `axis` argument (DISCONTINUOUS_LINEAR)
    int zcell;       // 3-D: the z frame is the cell frame of the bin keys (not shifted by dx/2)
    int xcell, ycell;  // 3-D: likewise the x and y frames
    int64_t s1, s2;  // strides of dims 1 and 2 (elements)
};

// The brick grid over stencil-anchor ("key") cells.  Bricks (8^3 cells in 3-D,
// 16^2 in 2-D) are numbered tile by tile (tiles of 4^NDIM bricks, tiles in
// linear order), Morton order inside a tile; an aligned 2^NDIM group of bricks
// (a spread "super-brick") therefore has 2^NDIM consecutive ids.
struct BinGeom {
    int ndim;
    int kmin[3];       // key cell of brick (0,0,0), cell (0,0,0)
    int nb[3];         // bricks per dim (multiple of 4)
    int nt[3];         // tiles per dim
    int nbricks;
    int shift;         // log2(cells per brick)
    double xlo[3];     // cell-frame x_lower of the patch
    double dx[3];
    int ilower[3];     // patch box lower
};

// 3-D column binning (le_sweep.hip).  Stencil-anchor ("key") cells are grouped
// into columns of COLX x COLY cells in (x, y); z is swept plane by plane.  Each
// (anchor plane, column) is split into NBAND bands by where the key cell sits
// in the column: xb = 0 / 2 if the stencil reaches the x-1 / x+1 column (1
// otherwise), yb likewise, band = 3*xb + yb.  Bucket = (z*ncol + col)*NBAND +
// band, col = cy*ncx + cx: the sorted list is z-major (every grid point sees its
// contributions in list order when the columns are swept in z), and the markers
// of a neighbouring column that reach a given column are a few contiguous bucket
// ranges.  Columns 0 and ncx-1 (rows 0 and ncy-1) are empty guards, so every
// real column has all eight neighbours.  nbuckets marks "outside".
constexpr int COLX = 32;
#ifndef IBTK_LE_COLY
#define IBTK_LE_COLY 16
#endif
constexpr int COLY = IBTK_LE_COLY;  // even: a 32 x COLY plane is whole wave rows
static_assert(COLY % 2 == 0 && COLY >= 8, "COLY: even, >= 8");
constexpr int NBAND = 9;
struct ColGeom {
    int org[3];     // absolute key cell of column (0,0) (a guard), plane 0
    int ext[3];     // key-cell extent covered: ncx*COLX, ncy*COLY, nz
    int ncx, ncy, nz, ncol;
    int nbuckets;   // nz * ncol * NBAND
};

// Diagnostic tuning of the 3-D sweeps (ibtk_le_ctx_tune); 0 = the default.
struct SweepTune {
    int seg_items = 0;     // sweep_segments' item target
    int split_target = 0;  // own markers above which a (column, segment) is cut (k_item_counts)
    int heavy = 0;         // own markers per piece above which an item is scheduled first (-1: never)
    int strip = 0;         // column rows per strip of the item order (0: default)
    int xcd_block = 0;     // light sweep items over the XCDs in blocks of this many table entries (1:
                           // round-robin; -1: one contiguous range per XCD; 0: the default, 8)
    int min_piece = 0;     // planes per sub-segment of a cut item, at least (0: the default, 8)
    int heavy_target = 0;  // a heavy item's pieces: own markers per piece (0: the default, le_sweep.hip HEAVY_TARGET)
    int heavy_min_piece = 0;  // ... and planes per piece, at least (0: HEAVY_MIN_PIECE)
    int heavy_first = 0;   // heavy items head the table (0, the default) or keep their place (-1)
    int interp3 = 0;       // 3-D interp of three components on one patch: 1 = one workgroup per item for
                           // all three (k_interp3: fewer bytes, measured slower); 0 = a workgroup per component
    int side_gather = 0;   // 3-D spread: the F gather on the side stream beside the candidate-stream
                           // rebuild (1), in line before the sweep (-1), or 0 (the default): on
                           // the side stream from 2^25 markers
};
// One 3-D sweep item: a patch, a column and its owned planes [p0, p1) (relative
// to the patch's cg.org[2]).
struct SweepItem {
    int col, p0, p1, patch;
};
// One patch of a level (3-D, ibtk_le_level_*): its column grid, its range of the
// level's bucket table and item enumeration, its cell frame, and its arrays.
struct PatchDesc {
    ColGeom cg;
    int bucket_base;  // first bucket of the patch in the level's table
    int ca_base_z;    // first column-anchor of the patch in the shifted-z frame (cs_off_z)
    int jbase;        // first (segment, column) pair of the patch (item table)
    int S, nseg;      // sweep segments
    double xlo[3];    // cell-frame x_lower
    int ilower[3];
    CompDesc comp[MAXC];
};

struct Params {
    BinGeom bg;
    ColGeom cg;                // 3-D column binning
    const unsigned* sorted_a;  // sorted position -> packed key cell (x | y << 16), relative to cg.org
    int S, nseg;               // sweep segment length (planes) and segments per column
    const PatchDesc* pd;       // 3-D level: per-patch descriptors (nullptr: one patch, cg/comp/bg above)
    int npatch;
    const int* entry_off;      // level: list entries of patch q are [entry_off[q], entry_off[q+1])
    int nbuckets_total;        // buckets of every patch (entries keyed >= it are outside)
    int njobs;                 // (segment, column) pairs of every patch
    int strip;                 // item order: column rows per strip (job_column)
    int ncut, cut[4];          // item table: extra cuts at these relative planes (the plane window's edges)
    int zmode, zlo, zhi;       // plane window (ibtk_le_ctx_set_plane_window): 0 every item, 1 the items
                               // whose planes lie in [zlo, zhi], 2 the others
    const SweepItem* items;    // 3-D sweep item table (k_item_write)
    const int* items_skip;     // k_item_counts / k_item_write: nothing to do when *items_skip == 0 (a
                               // re-binning that moved nothing leaves the bucket starts, so the table, as they were)
    const int* nitems;         // device: its length, then the count of heavy items heading it
    int item_bound;            // host: an upper bound of the length (the launch grid)
    SweepTune tune;
    int ncomp;
    CompDesc comp[MAXC];
    int Q_depth;
    double h3;                 // dx0*dx1[*dx2], associated as the Fortran does
    double K6;                 // IB_6 parameter K
    const double* X;           // AoS positions
    const int* indices;        // list entry -> marker (nullptr: identity)
    const double* Xshift;      // list entry -> shift[NDIM] (nullptr: zero)
    const int* sorted_l;       // sorted position -> list entry
    const int* sorted_s;       // sorted position -> marker index
    const double* sorted_X;    // sorted position -> X(s) + Xshift(l) [NDIM]
    const double* const* sorted_X_ref;  // 3-D: device cell naming the current sorted positions (or null: sorted_X)
    const unsigned* sorted_key;
    const int* plane_start;    // nbricks*B + 1 offsets into the sorted list: bucket = key >> (shift - log2 B)
                               // (brick b's entries are [plane_start[b*B], plane_start[(b+1)*B]))
    const int* cand_off;       // spread: (super-brick, class) candidate lists: offsets, items*NCLS + 1
    const int* cand_idx;       // spread: candidate sorted positions, canonical order per super-brick
    const int* cs_off;         // 3-D spread: candidate stream offsets per column-anchor (launch_cand_stream)
    const int* cs_pos;         // 3-D spread: the candidate stream (sorted positions)
    int cs_total;              // its length
    const int* cs_off_z;       // closed-form kernels: the stream's boundaries per anchor of the frame
                               // shifted by -dz/2 in z (side-z, node, x/y-edge components; k_cand_write)
    int cs_rint;               // the spread's stencils anchor by rint (IB_4), not NINT
    const int* cs_zflip;       // with cs_off_z and items_skip: == cs_epoch when a shifted-z anchor changed
    int cs_epoch;              //     in the last re-binning (RebinBufs::zst, epoch)
    const int* nentries_dev;   // device copy of the list length
    const double* Qin;         // spread: marker values
    const double* sorted_F;    // spread: Qin gathered in sorted order, [comp][sorted position]
    const double* ds;          // spread: per-marker weight (nullptr: none); sorted_F = Qin * ds
    int nsorted;               // list length
    double* Qout;              // interp: marker values
    const int* qdst;           // interp: per sorted entry, the marker whose Q it writes, or -1 when a later
                               // list entry of the same marker writes it (the Fortran's sequential l-loop
                               // overwrites: the last occurrence wins); nullptr = sorted_s (no duplicates)
    int* err;                  // device error word (0 = fine)
    double* sink;              // 64 doubles: the store target of masked-off lanes (branch-free stores)
    const int* n_dev = nullptr;  // bin: the list's length on the device (entries beyond it binned outside)
    unsigned long long* stamps = nullptr;  // diagnostic phase clocks (nullptr: off)
    unsigned long long* nadd = nullptr;    // spread: [ds_add_f64 wave-instructions, lane adds] issued (nullptr: not counted)
    int zero_first = 0;  // 3-D spread: the arrays start from 0 (every point, ghosts included), not their values
    int zero_ghosts = 0; // 3-D spread: the ghost points (outside the data box) start from 0, the others from their values
    int iper[3] = {0, 0, 0};  // 3-D interp: read the ghost points of the ghost box at their periodic image in
                              // these dims (ibtk_le_fill_interp: the periodic ghost fill fused in)
    int comp0 = 0;       // 3-D spread: a launch's components are comp[comp0 .. comp0 + ncomp)
    // 3-D level interp with the level's ghost fill fused in (ibtk_le_level_fill_interp): a
    // ghost point is read where the fill would copy it from -- the neighbour patch owning
    // its cell (27 directions), at the same global index.  Component c's arrays of every
    // patch lie in one window below 2 GB; record (c * npatch + q) of lvl_nbr (32 int2):
    // [dir] = {byte offset of the supplying array in the window, 1 if it is the neighbour
    // in dir (index mapped by -dir n), 0 if none (own array, as is)}, [27] = the window's
    // base (lo, hi), [28].x = its length in bytes.
    const int2* lvl_nbr = nullptr;
    int lvl_n[3] = {0, 0, 0};  // cells per patch and dim
};

// Host-side launchers (le_kernels.hip).
hipError_t launch_bin(int ndim, int kernel, const Params& p, int n, unsigned* keys, int* vals, hipStream_t s);
hipError_t launch_brick_start(const unsigned* keys, int n, int nbricks, int shift, int* bs, hipStream_t s);
hipError_t launch_gather_sorted(int ndim, const Params& p, int n, int* sorted_s, double* sorted_X, hipStream_t s);
hipError_t launch_interp(int ndim, int kernel, const Params& p, int n, hipStream_t s, hipEvent_t ev0,
                         hipEvent_t ev1);
hipError_t launch_spread(int ndim, int kernel, const Params& p, hipStream_t s, hipEvent_t ev0, hipEvent_t ev1);
hipError_t launch_cand(int ndim, int kernel, const Params& p, bool write, int* counts_or_offs, int* out, hipStream_t s);
int cand_classes(int ndim, int kernel);  // candidate classes per super-brick
hipError_t launch_mark(int ndim, int kernel, const Params& p, int n, unsigned char** masks, hipStream_t s);
hipError_t launch_sort(void* temp, size_t& temp_bytes, const unsigned* kin, unsigned* kout, const int* vin,
                       int* vout, int n, int end_bit, hipStream_t s);
hipError_t launch_scan(void* temp, size_t& temp_bytes, const int* in, int* out, int n, hipStream_t s);
hipError_t launch_suffix_min(void* temp, size_t& temp_bytes, const int* in, int* out, int n, hipStream_t s);

// 3-D column sweep (le_sweep.hip)
hipError_t launch_bin_col(int kernel, const Params& p, int n, unsigned* keys, int* vals, hipStream_t s);
// Incremental re-binning of a binned list at new positions (ibtk_le_markers_rebin,
// le_sweep.hip k_rekey .. k_rebin_scatter).  nb = buckets (the outside bucket is nb);
// per-bucket arrays hold nb + 2 ints, per-word arrays nw + 1 (nw = ceil(n / 32)).
struct RebinBufs {
    int n, nb, nw;
    const unsigned* kold;  // the old sorted keys (sorted_key, read before the scatter rewrites it)
    const int* lsorted;    // the old sorted_l (read by k_rekey)
    unsigned* knew;        // new key per old sorted position
    int* lold;             // copy of the old sorted_l
    unsigned* mbits;       // mover flag per old sorted position, 32 per word (word nw stays 0)
    int* wcnt;             // movers per word (entry nw stays 0)
    int* wpre;             // its exclusive prefix (wpre[nw] = movers)
    int* cin;              // movers into bucket b (0 on entry; consumed back to 0)
    int* cout;             // movers out of bucket b (0 on entry; reset)
    int* d;                // scratch: per block of buckets, the sums of (cin - cout, cin) as int2
    int* dpre;             // (unused)
    int* mstart;           // exclusive prefix of cin: bucket b's movers are mlist[mstart[b] .. mstart[b+1])
    int* mlist;            // the movers' l, per bucket sorted by l
    int* scratch;          // long lists' sort
    int* nbig;             // long lists queued (zeroed before)
    int* big;
    const int* os;         // old bucket starts (plane_start)
    int* ns;               // new bucket starts
    int* sorted_l;
    unsigned* sorted_key;
    int* sorted_s;
    double** xcur;          // the current sorted-position buffer (xa or xb; le_sweep.hip rebin_other)
    double* xa;
    double* xb;
    int* order_gen;         // bumped when something moved (the order changed; nullable)
    unsigned* zbits;        // shifted-z anchor parities per sorted position (nw + 1 words; k_rekey)
    int* zst;               // [0] zbits are in the current order, [1] = epoch: a parity changed
    int epoch;              // this re-binning's number (nonzero)
};
hipError_t launch_set_xcur(double** xcur, double* x, hipStream_t s);
hipError_t launch_rekey(int kernel, const Params& p, const RebinBufs& r, hipStream_t s);

hipError_t launch_rebin_copy(int kernel, const Params& p, const RebinBufs& r, hipStream_t s);
hipError_t launch_rebin_starts(const RebinBufs& r, hipStream_t s);  // uses r.d as the block sums (int2)
hipError_t launch_rebin_movers(const RebinBufs& r, hipStream_t s);
hipError_t launch_rebin_scatter(const Params& p, const RebinBufs& r, hipStream_t s);
// z-slab migration classes (le_aux.hip)
struct SlabMig {
    double L[3];
    double dz;
    int Nz, nz, P, rank;
    const int* n_dev;  // nullptr: all M rows; else the rows in use (a fixed-capacity list)
};
// Fixed-capacity migration (no host sync).  rows: [M][D] doubles; order/counts from
// the partition ([stay | down | up | far]).  pack: the down / up leavers into
// send_down / send_up (send_cap rows each); unpack: out = stayers in order, then
// from_down[0:rc[0]], then from_up[0:rc[1]]; *n_out = their number.  Overflow
// (leavers > send_cap, far markers, arrivals past out_cap) sets err bit 8.
hipError_t launch_mig_pack(const double* rows, int D, const int* order, const int* counts, int send_cap,
                           double* send_down, double* send_up, int* err, hipStream_t s);
hipError_t launch_mig_unpack(const double* rows, int D, const int* order, const int* counts, const int* rc,
                             const double* from_down, const double* from_up, int send_cap, double* out, int out_cap,
                             int* n_out, int* err, hipStream_t s);
hipError_t launch_slab_update_partition(int scheme, long M, double dt, const double* X, const double* U0,
                                        const double* U1, double* Xn, const SlabMig& g, unsigned char* cls,
                                        int* bcount, int* boff, void* temp, size_t& temp_bytes, int* order,
                                        int* counts, hipStream_t s);
hipError_t launch_position_update(int scheme, long n, double dt, const double* X, const double* U0, const double* U1,
                                  double* Xn, hipStream_t s);
hipError_t launch_gather_col(int kernel, const Params& p, int n, int* sorted_s, double* sorted_X,
                             const unsigned* sorted_key, int nbuckets, int* bucket_start, hipStream_t s);
hipError_t launch_interp_sweep(int kernel, const Params& p, int n, hipStream_t s, hipEvent_t ev0, hipEvent_t ev1);
// gather = false: the spread values (sorted_F) were gathered already (launch_gather_F, on
// the context's side stream while the candidate stream was rebuilt)
hipError_t launch_spread_sweep(int kernel, const Params& p, hipStream_t s, hipEvent_t ev0, hipEvent_t ev1,
                               bool gather = true);
hipError_t launch_gather_F(const Params& p, hipStream_t s);
void sweep_segments(const ColGeom& cg, int& S, int& nseg, int seg_items, bool level);
hipError_t launch_item_table(int kernel, const Params& p, int target, int heavy, int* nsub, int* start, SweepItem* tab, int* ntot,
                             void* temp, size_t temp_bytes, hipStream_t s);
// the spread's candidate stream of a 3-D column binning: cnt[ncl + 1] (cnt[ncl] = 0 on entry),
// off[ncl + 1] (off[ncl] = the length), pos[length]; p.items_skip as for the item table.
// p.cs_off_z set (closed-form kernels): each anchor's candidates split by their shifted-z
// anchor and p.cs_off_z[Σ ncol (nz + 1) + 1] written (k_cand_write; no skip)
// total: a device u64 for the stream's length in 64 bits (a stream longer than p.cs_total
// raises device flag 16 and is not written)
hipError_t launch_cand_stream(const Params& p, int ncl, int* cnt, int* off, int* pos, void* temp, size_t temp_bytes,
                              unsigned long long* total, hipStream_t s);

// Periodic helpers
struct GhostDesc {
    double* u;
    int lo[3], hi[3];     // ghost box
    int ilo[3], ihi[3];   // unique (interior) index range per dim
    int64_t s1, s2;
};
constexpr int GSET = 4;  // arrays per ghost launch
struct GhostSet {
    GhostDesc g[GSET];
};
// every pass covers all n arrays (GSET per launch)
hipError_t launch_fill_periodic(int ndim, const GhostDesc* g, int n, const int* periodic, hipStream_t s);
hipError_t launch_fold_periodic(int ndim, const GhostDesc* g, int n, const int* periodic, hipStream_t s);
hipError_t launch_zero_ghosts(int ndim, const GhostDesc* g, int n, hipStream_t s);

struct ImageDesc {
    int ndim;
    double xlo[3], xup[3], dx[3];
    int ilo[3], ihi[3];
    int ghost;
    int periodic[3];
    int filter;           // 1: emit (s, 0) iff the cell lies in [flo, fhi] (no images)
    int flo[3], fhi[3];
    int which;            // images: 0 every cell of the ghost box, 1 patch-box cells, 2 the others
    int sub;              // 1: images only in cells of [slo, shi] (buildLocalIndices' box, LEInteractor.cpp:3070-3106)
    int slo[3], shi[3];
};
hipError_t launch_cell_keys(const ImageDesc& d, const double* X, int n, unsigned ncells, unsigned* keys, int* vals,
                            int* inside, hipStream_t s);
hipError_t launch_image_count(const ImageDesc& d, const double* X, int n, int* counts, hipStream_t s);
// interp with duplicate list entries: qdst[e] (see Params::qdst); *ndup (device) counts the -1s
hipError_t launch_max_index(const int* idx, int n, int* out, hipStream_t s);
hipError_t launch_dedup(const int* indices, const int* sorted_l, const int* sorted_s, int n, int* last, int* qdst,
                        int* ndup, hipStream_t s);
hipError_t launch_image_write(const ImageDesc& d, const double* X, int n, const int* offsets, int* idx,
                              double* xshift, unsigned* cellkey, int* cells, int capacity, hipStream_t s);
// small helpers of the reference-ordered lists (le_aux.hip)
hipError_t launch_iota(int* v, int n, hipStream_t s);
hipError_t launch_sum64(const int* v, int n, unsigned long long* out, hipStream_t s);
// out[i] = key_of(src[perm[i]]): mode 0 lag[idx[perm[i]]] (lag null: idx[perm[i]]), mode 1 keys[perm[i]]
hipError_t launch_perm_keys(int mode, const int* perm, const int* idx, const int* lag, const unsigned* keys, int n,
                            unsigned* out, hipStream_t s);
hipError_t launch_perm_list(const int* perm, const int* idx, const double* xs, const int* cells, int ndim, int n,
                            int* idx_out, double* xs_out, int* cells_out, hipStream_t s);
// list entries kept where flag[i] (pos = exclusive scan of flag): out[pos[i]] = in[i]
hipError_t launch_compact_list(const int* flag, const int* pos, const int* idx, const double* xs, const int* cells,
                               int ndim, int n, int* idx_out, double* xs_out, int* cells_out, hipStream_t s);
// flag[i] = cells[ndim i ..] lies in [lo, hi]
hipError_t launch_in_box_flags(const int* cells, int ndim, int n, const int* lo, const int* hi, int* flag,
                               hipStream_t s);
// node distribution: region/cell keys (local cells, then the ghost box's others, then out)
hipError_t launch_node_keys(const ImageDesc& d, const double* X, int n, unsigned* keys, hipStream_t s);
// unique by (key, lag) over the sorted order: flag[i] = 1 for a first occurrence
hipError_t launch_unique_flags(const unsigned* skeys, const int* sorder, const int* lag, int n, int* flag,
                               hipStream_t s);
hipError_t launch_compact(const int* sorder, const int* flag, const int* pos, const unsigned* skeys,
                          unsigned local_end, unsigned ghost_end, int n, int* out, int* counts, hipStream_t s);

// Level numbering (ibtk_le_level_node_distribution, le_aux.hip): the local patches
// of one level, equal boxes of n cells per dim aligned to a tiling from `org`; a
// table of nt tiles maps a tile to the patch's rank in the level's patch order
// (-1: not a local patch).  Cells by getCellIndex in the domain frame.
struct LevelNum {
    int ndim;
    double xlo[3], xup[3], dx[3];  // domain frame
    int dom_lo[3], dom_hi[3];      // domain cells (periodic images shift by its extent)
    int periodic[3];
    int n[3];                      // cells per patch
    int org[3];                    // lower cell of tile (0, 0, 0)
    int nt[3];                     // tiles per dim of the table
    int g;                         // ghost width of the patches' index data
    float rn[3];                   // 1 / n[k] (le_aux.hip lfloordiv: the quotient's estimate)
};
// cls[s]: 0 the marker lies in a local patch (key_local = patch rank * cells per
// patch + its cell's box index), 1 only in ghost cells (key_ghost = the first
// occurrence: patch rank * ghost-box cells + ghost-box index of its (image) cell),
// 2 neither.  lkey = key_local for cls 0, else 0xffffffff; ckey = 0 for cls 0, 1 +
// key_ghost for cls 1, 0xffffffff for cls 2.
hipError_t launch_level_node_keys(const LevelNum& L, const int* tab, const double* X, int n, unsigned* lkey,
                                  unsigned* ckey, hipStream_t s);
// A level's index lists (ibtk_le_level_index_lists): per marker its interior key (patch *
// patch cells + box index; 0xffffffff outside every local patch box) and ghost-box entry
// count; then its entries at goff[s] (key = patch * ghost-box cells + ghost-box index of the
// image's cell, id = the entry's own index, the marker, the image 0 .. 26); the entries taken
// in sorted order (sid) out as marker indices and periodic shifts; off[q] = first sorted key
// >= q * per, q = 0 .. npatch.
// (bypatch: the keys are the patch alone, npatch for none -- marker order within a patch)
hipError_t launch_level_list_keys(const LevelNum& L, const int* tab, const double* X, int n, unsigned* ikey,
                                  int* gcnt, int bypatch, int npatch, hipStream_t s);
hipError_t launch_level_list_write(const LevelNum& L, const int* tab, const double* X, int n, const int* goff,
                                   unsigned* gkey, int* gid, int* gsrc, int* gimg, int bypatch, hipStream_t s);
hipError_t launch_level_list_out(const LevelNum& L, const int* sid, const int* gsrc, const int* gimg, int total,
                                 int* idx, double* xs, hipStream_t s);
hipError_t launch_key_offsets(const unsigned* skeys, int n, unsigned per, int npatch, int* off, hipStream_t s);
// A level's interp restricted to its interior lists (ibtk_le_level_select_interior):
// owner[s] = max patch whose interior list names marker s (owner pre-filled with -1);
// then per sorted entry e of the binned lists: qin[e] = s if owner[s] is the entry's
// patch and the entry is unshifted, else -1; found[block] counts the block's kept entries.
// Marker indices outside [0, n_markers) (in either list) are not dereferenced: err bit 4.
// gs: the selection cache {order generation, generation of the selection} (nullable):
// equal, and the kernels return at once; launch_sel_mark records the selection's
hipError_t launch_interior_owner(const int* int_off, int npatch, const int* int_idx, int n_int, int n_markers,
                                 int* owner, int* err, const int* gs, hipStream_t s);
hipError_t launch_interior_targets(const int* sorted_l, const int* sorted_s, const int* entry_off, int npatch,
                                   const double* xshift, const int* owner, int n_markers, int n, int* qin, int* found,
                                   int* err, const int* gs, hipStream_t s);
hipError_t launch_sel_mark(int* gs, hipStream_t s);
struct WrapBox {
    double lo[3], hi[3];
    int per[3];
    int ndim;
};
hipError_t launch_wrap_positions(const WrapBox& w, long long n, double* X, hipStream_t s);
// sum(count[0:ncount]) != expect: atomicOr(err, bit)
// USER_DEFINED kernel function (LEInteractor::userDefinedInterpolate / Spread,
// LEInteractor.cpp:3141-3393): the host evaluates the user's phi(r) for every list
// entry (phi is a host function pointer); the device sums and spreads.  Per entry
// l and dim d: the clipped stencil's first index lo[3 l + d], its length cnt[3 l + d]
// and its weights w[(3 l + d) S + i].
struct UserDesc {
    CompDesc cd;
    int ndim, S, n;
    const int* lo;
    const int* cnt;
    const double* w;
    const int* sidx;   // entry -> marker
    const int* last;   // interp: 1 if the entry is the last one naming its marker (it writes Q)
    const double* Q;   // spread: marker values
    double* Qout;      // interp: marker values
    int Q_depth;
    double dxprod;     // spread: dx0 dx1 [dx2], associated as the reference does
};
hipError_t launch_user_gather(const double* X, const int* indices, const double* Xshift, int n, int ndim, double* Xraw,
                              double* Xsh, int* sidx, hipStream_t s);
hipError_t launch_user_interp(const UserDesc& u, hipStream_t s);
// spread, deterministic: per-point contributions keyed by array offset, stably sorted,
// then summed point by point in list order (the reference's sequential l-loop)
hipError_t launch_user_contrib(const UserDesc& u, unsigned* keys, int* vals, double* contrib, hipStream_t s);
hipError_t launch_user_segsum(const UserDesc& u, const unsigned* skeys, const int* svals, const double* contrib,
                              int ncontrib, hipStream_t s);
constexpr int CHECK_STRIPES = 64;  // counters k_interior_targets adds its block counts into
hipError_t launch_check_count(const int* count, int ncount, int expect, int* err, int bit, hipStream_t s,
                              const int* gs = nullptr);
// out[i * depth + k] = in[order[i] * depth + k]
hipError_t launch_rows_gather(const int* order, int n, const double* in, int depth, double* out, hipStream_t s);
// flag[i] = entry i of the (lag, ckey)-sorted list is the first of its lag run and not local
hipError_t launch_nonlocal_flags(const unsigned* sckey, const int* sorder, const int* lag, int n, int* flag,
                                 hipStream_t s);
// out[i] = keys[idx[i]]
hipError_t launch_take_keys(const unsigned* keys, const int* idx, int n, unsigned* out, hipStream_t s);

// Ghost fill of a level of equal patches tiling a box (le_aux.hip): every ghost
// point of every patch array takes the value of the patch that owns the point
// (wrapped in periodic dims).
struct LevelTiling {
    int n[3];        // cells per patch and dim
    int ntile[3];    // patches per dim
    int dom_lo[3];   // lower cell of the tiled box
    int g;           // ghost width
    int periodic[3];
    int ncomp;       // arrays per patch (side: 3, cell/node depth slices: 1)
    int side;        // 1: side-centred (array a has one extra face along a)
};
hipError_t launch_level_fill(const LevelTiling& t, int npatch, const int* tile_of_patch, const int* patch_of_tile,
                             double* const* arrays, int depth, hipStream_t s);
hipError_t launch_level_zero(double* const* arrays, const long long* count, int narr, long long max_count,
                             hipStream_t s);

// Physical-boundary ghost operators on one side-centred patch (le_bdry.hip)
struct BdSide {
    double* u[3];
    int lo[3][3];          // ghost-box lower corner of component c
    int64_t s1[3], s2[3];  // strides of component c
    int ilo[3], ihi[3];    // patch cell box (0 past ndim)
    double dx[3];
    int g, ndim;
};
struct BdCoef {
    double a, b, g;
};
// coef[c * 2 ndim + loc]: Robin a, b, g of component c on face loc
hipError_t launch_phys_bdry_side(const BdSide& P, const int* phys, const BdCoef* coef, int adjoint, hipStream_t s);

}  // namespace ibtk_le

// Internal entry used by the Fortran shims (skips the LEInteractor-level ghost check).
struct ibtk_le_ctx_s;
struct ibtk_le_markers_s;
struct ibtk_le_patch_geom_s;
namespace ibtk_le {
int interp_impl(ibtk_le_ctx_s* ctx, ibtk_le_markers_s* m, int kernel, int centering, int axis, const void* geom,
                const double* const* q_dev, int q_depth, double* Q_dev, int Q_depth, const double* X_dev,
                bool check_ghosts, const int* iper = nullptr);
}  // namespace ibtk_le
