/* le_oracle.h -- CPU restatement of the reference Fortran kernels.
 * TEST INFRASTRUCTURE ONLY: see the header comment of le_oracle.c. */
#ifndef LE_ORACLE_H
#define LE_ORACLE_H

#ifdef __cplusplus
extern "C" {
#endif

/* Kernel ids: same numbering as include/ibtk_le.h (IBTK_LE_KERNEL_*). */
enum {
    LE_PIECEWISE_CONSTANT = 0,
    LE_DISCONTINUOUS_LINEAR = 1,
    LE_PIECEWISE_LINEAR = 2,
    LE_PIECEWISE_CUBIC = 3,
    LE_IB_3 = 4,
    LE_IB_4 = 5,
    LE_IB_4_W8 = 6,
    LE_IB_6 = 7,
    LE_BSPLINE_4 = 8
};

int ora_stencil_size(int kernel);
int ora_lagrangian_floor(double x);
double ora_piecewise_cubic_delta(double r);
double ora_ib_3_delta(double r);
int ora_closed_form_weights(int kernel, double X_o_dx, int ilower, double* w);

/* One depth-`depth` call of lagrangian_<kernel>_interp{2,3}d.  `axis` is only
 * read by DISCONTINUOUS_LINEAR.  Returns 0 on success. */
int ora_interp(int kernel, int ndim, const double* dx, const double* x_lower, int depth, int axis, const int* ilower,
               const int* iupper, const int* nugc, const double* u, const int* indices, const double* Xshift,
               int nindices, const double* X, double* V);

/* One call of lagrangian_<kernel>_spread{2,3}d: u += S V, in list order. */
int ora_spread(int kernel, int ndim, const double* dx, const double* x_lower, int depth, int axis, const int* ilower,
               const int* iupper, const int* nugc, double* u, const int* indices, const double* Xshift, int nindices,
               const double* X, const double* V);

/* CartSideRobinPhysBdryOp on one side-centred patch (le_bdry_oracle.c):
 * adjoint = 0 fills the physical-boundary ghosts (setPhysicalBoundaryConditions),
 * adjoint = 1 folds them back (accumulateFromPhysicalBoundaryData).  u0..u2 are
 * the ghosted side arrays of axes 0..ndim-1 (uniform ghost width gcw); phys[loc]
 * flags face loc = 2 d + upper as physical; coefficient [c * 2 ndim + loc] is
 * the Robin a/b/g of component c on face loc. */
int ora_phys_bdry_side(int ndim, const int* ilower, const int* iupper, int gcw, const double* dx, double* u0,
                       double* u1, double* u2, const int* phys, const double* acoef, const double* bcoef,
                       const double* gcoef, int adjoint);

/* USER_DEFINED (LEInteractor.cpp:3141-3393): phi a host kernel function, S its stencil size */
int ora_user_call(double (*phi)(double), int S, int spread, int ndim, const double* dx, const double* x_lower,
                  int depth, const int* ilower, const int* iupper, const int* nugc, double* u, const int* indices,
                  const double* Xshift, int nindices, const double* X, double* V);

#ifdef __cplusplus
}
#endif
#endif
