/*
 * ibtk_le_fortran.h -- the Fortran-symbol drop-in entry points.
 *
 * These are the exact symbols and argument lists that IBTK's LEInteractor.cpp
 * declares in its extern "C" block (ibtk/src/lagrangian/LEInteractor.cpp:68-619,
 * IBTK_FC_FUNC_ = lowercase name + trailing underscore) and that
 * ibtk/src/lagrangian/fortran/lagrangian_interaction{2,3}d.f.m4 define.  Linking
 * libibtk_le.so in place of those Fortran objects reroutes every
 * LEInteractor::interpolate/spread call to the MI355X kernels.  All arguments are
 * host pointers, scalars by reference (Fortran convention).  x_upper is unused,
 * as in the Fortran.  DISCONTINUOUS_LINEAR takes `axis` after `depth`.
 */
#ifndef IBTK_LE_FORTRAN_H
#define IBTK_LE_FORTRAN_H

#ifdef __cplusplus
extern "C" {
#endif

/* PIECEWISE_CONSTANT -- lagrangian_interaction3d.f.m4 / lagrangian_interaction2d.f.m4 */
void lagrangian_piecewise_constant_interp3d_(const double* dx, const double* x_lower, const double* x_upper, const int* depth, const int* ilower0, const int* iupper0, const int* ilower1, const int* iupper1, const int* ilower2, const int* iupper2, const int* nugc0, const int* nugc1, const int* nugc2, const double* u, const int* indices, const double* Xshift, const int* nindices, const double* X, double* V);
void lagrangian_piecewise_constant_spread3d_(const double* dx, const double* x_lower, const double* x_upper, const int* depth, const int* indices, const double* Xshift, const int* nindices, const double* X, const double* V, const int* ilower0, const int* iupper0, const int* ilower1, const int* iupper1, const int* ilower2, const int* iupper2, const int* nugc0, const int* nugc1, const int* nugc2, double* u);
void lagrangian_piecewise_constant_interp2d_(const double* dx, const double* x_lower, const double* x_upper, const int* depth, const int* ilower0, const int* iupper0, const int* ilower1, const int* iupper1, const int* nugc0, const int* nugc1, const double* u, const int* indices, const double* Xshift, const int* nindices, const double* X, double* V);
void lagrangian_piecewise_constant_spread2d_(const double* dx, const double* x_lower, const double* x_upper, const int* depth, const int* indices, const double* Xshift, const int* nindices, const double* X, const double* V, const int* ilower0, const int* iupper0, const int* ilower1, const int* iupper1, const int* nugc0, const int* nugc1, double* u);

/* DISCONTINUOUS_LINEAR -- lagrangian_interaction3d.f.m4 / lagrangian_interaction2d.f.m4 */
void lagrangian_discontinuous_linear_interp3d_(const double* dx, const double* x_lower, const double* x_upper, const int* depth, const int* axis, const int* ilower0, const int* iupper0, const int* ilower1, const int* iupper1, const int* ilower2, const int* iupper2, const int* nugc0, const int* nugc1, const int* nugc2, const double* u, const int* indices, const double* Xshift, const int* nindices, const double* X, double* V);
void lagrangian_discontinuous_linear_spread3d_(const double* dx, const double* x_lower, const double* x_upper, const int* depth, const int* axis, const int* indices, const double* Xshift, const int* nindices, const double* X, const double* V, const int* ilower0, const int* iupper0, const int* ilower1, const int* iupper1, const int* ilower2, const int* iupper2, const int* nugc0, const int* nugc1, const int* nugc2, double* u);
void lagrangian_discontinuous_linear_interp2d_(const double* dx, const double* x_lower, const double* x_upper, const int* depth, const int* axis, const int* ilower0, const int* iupper0, const int* ilower1, const int* iupper1, const int* nugc0, const int* nugc1, const double* u, const int* indices, const double* Xshift, const int* nindices, const double* X, double* V);
void lagrangian_discontinuous_linear_spread2d_(const double* dx, const double* x_lower, const double* x_upper, const int* depth, const int* axis, const int* indices, const double* Xshift, const int* nindices, const double* X, const double* V, const int* ilower0, const int* iupper0, const int* ilower1, const int* iupper1, const int* nugc0, const int* nugc1, double* u);

/* PIECEWISE_LINEAR -- lagrangian_interaction3d.f.m4 / lagrangian_interaction2d.f.m4 */
void lagrangian_piecewise_linear_interp3d_(const double* dx, const double* x_lower, const double* x_upper, const int* depth, const int* ilower0, const int* iupper0, const int* ilower1, const int* iupper1, const int* ilower2, const int* iupper2, const int* nugc0, const int* nugc1, const int* nugc2, const double* u, const int* indices, const double* Xshift, const int* nindices, const double* X, double* V);
void lagrangian_piecewise_linear_spread3d_(const double* dx, const double* x_lower, const double* x_upper, const int* depth, const int* indices, const double* Xshift, const int* nindices, const double* X, const double* V, const int* ilower0, const int* iupper0, const int* ilower1, const int* iupper1, const int* ilower2, const int* iupper2, const int* nugc0, const int* nugc1, const int* nugc2, double* u);
void lagrangian_piecewise_linear_interp2d_(const double* dx, const double* x_lower, const double* x_upper, const int* depth, const int* ilower0, const int* iupper0, const int* ilower1, const int* iupper1, const int* nugc0, const int* nugc1, const double* u, const int* indices, const double* Xshift, const int* nindices, const double* X, double* V);
void lagrangian_piecewise_linear_spread2d_(const double* dx, const double* x_lower, const double* x_upper, const int* depth, const int* indices, const double* Xshift, const int* nindices, const double* X, const double* V, const int* ilower0, const int* iupper0, const int* ilower1, const int* iupper1, const int* nugc0, const int* nugc1, double* u);

/* PIECEWISE_CUBIC -- lagrangian_interaction3d.f.m4 / lagrangian_interaction2d.f.m4 */
void lagrangian_piecewise_cubic_interp3d_(const double* dx, const double* x_lower, const double* x_upper, const int* depth, const int* ilower0, const int* iupper0, const int* ilower1, const int* iupper1, const int* ilower2, const int* iupper2, const int* nugc0, const int* nugc1, const int* nugc2, const double* u, const int* indices, const double* Xshift, const int* nindices, const double* X, double* V);
void lagrangian_piecewise_cubic_spread3d_(const double* dx, const double* x_lower, const double* x_upper, const int* depth, const int* indices, const double* Xshift, const int* nindices, const double* X, const double* V, const int* ilower0, const int* iupper0, const int* ilower1, const int* iupper1, const int* ilower2, const int* iupper2, const int* nugc0, const int* nugc1, const int* nugc2, double* u);
void lagrangian_piecewise_cubic_interp2d_(const double* dx, const double* x_lower, const double* x_upper, const int* depth, const int* ilower0, const int* iupper0, const int* ilower1, const int* iupper1, const int* nugc0, const int* nugc1, const double* u, const int* indices, const double* Xshift, const int* nindices, const double* X, double* V);
void lagrangian_piecewise_cubic_spread2d_(const double* dx, const double* x_lower, const double* x_upper, const int* depth, const int* indices, const double* Xshift, const int* nindices, const double* X, const double* V, const int* ilower0, const int* iupper0, const int* ilower1, const int* iupper1, const int* nugc0, const int* nugc1, double* u);

/* IB_3 -- lagrangian_interaction3d.f.m4 / lagrangian_interaction2d.f.m4 */
void lagrangian_ib_3_interp3d_(const double* dx, const double* x_lower, const double* x_upper, const int* depth, const int* ilower0, const int* iupper0, const int* ilower1, const int* iupper1, const int* ilower2, const int* iupper2, const int* nugc0, const int* nugc1, const int* nugc2, const double* u, const int* indices, const double* Xshift, const int* nindices, const double* X, double* V);
void lagrangian_ib_3_spread3d_(const double* dx, const double* x_lower, const double* x_upper, const int* depth, const int* indices, const double* Xshift, const int* nindices, const double* X, const double* V, const int* ilower0, const int* iupper0, const int* ilower1, const int* iupper1, const int* ilower2, const int* iupper2, const int* nugc0, const int* nugc1, const int* nugc2, double* u);
void lagrangian_ib_3_interp2d_(const double* dx, const double* x_lower, const double* x_upper, const int* depth, const int* ilower0, const int* iupper0, const int* ilower1, const int* iupper1, const int* nugc0, const int* nugc1, const double* u, const int* indices, const double* Xshift, const int* nindices, const double* X, double* V);
void lagrangian_ib_3_spread2d_(const double* dx, const double* x_lower, const double* x_upper, const int* depth, const int* indices, const double* Xshift, const int* nindices, const double* X, const double* V, const int* ilower0, const int* iupper0, const int* ilower1, const int* iupper1, const int* nugc0, const int* nugc1, double* u);

/* IB_4 -- lagrangian_interaction3d.f.m4 / lagrangian_interaction2d.f.m4 */
void lagrangian_ib_4_interp3d_(const double* dx, const double* x_lower, const double* x_upper, const int* depth, const int* ilower0, const int* iupper0, const int* ilower1, const int* iupper1, const int* ilower2, const int* iupper2, const int* nugc0, const int* nugc1, const int* nugc2, const double* u, const int* indices, const double* Xshift, const int* nindices, const double* X, double* V);
void lagrangian_ib_4_spread3d_(const double* dx, const double* x_lower, const double* x_upper, const int* depth, const int* indices, const double* Xshift, const int* nindices, const double* X, const double* V, const int* ilower0, const int* iupper0, const int* ilower1, const int* iupper1, const int* ilower2, const int* iupper2, const int* nugc0, const int* nugc1, const int* nugc2, double* u);
void lagrangian_ib_4_interp2d_(const double* dx, const double* x_lower, const double* x_upper, const int* depth, const int* ilower0, const int* iupper0, const int* ilower1, const int* iupper1, const int* nugc0, const int* nugc1, const double* u, const int* indices, const double* Xshift, const int* nindices, const double* X, double* V);
void lagrangian_ib_4_spread2d_(const double* dx, const double* x_lower, const double* x_upper, const int* depth, const int* indices, const double* Xshift, const int* nindices, const double* X, const double* V, const int* ilower0, const int* iupper0, const int* ilower1, const int* iupper1, const int* nugc0, const int* nugc1, double* u);

/* IB_4_W8 -- lagrangian_interaction3d.f.m4 / lagrangian_interaction2d.f.m4 */
void lagrangian_ib_4_w8_interp3d_(const double* dx, const double* x_lower, const double* x_upper, const int* depth, const int* ilower0, const int* iupper0, const int* ilower1, const int* iupper1, const int* ilower2, const int* iupper2, const int* nugc0, const int* nugc1, const int* nugc2, const double* u, const int* indices, const double* Xshift, const int* nindices, const double* X, double* V);
void lagrangian_ib_4_w8_spread3d_(const double* dx, const double* x_lower, const double* x_upper, const int* depth, const int* indices, const double* Xshift, const int* nindices, const double* X, const double* V, const int* ilower0, const int* iupper0, const int* ilower1, const int* iupper1, const int* ilower2, const int* iupper2, const int* nugc0, const int* nugc1, const int* nugc2, double* u);
void lagrangian_ib_4_w8_interp2d_(const double* dx, const double* x_lower, const double* x_upper, const int* depth, const int* ilower0, const int* iupper0, const int* ilower1, const int* iupper1, const int* nugc0, const int* nugc1, const double* u, const int* indices, const double* Xshift, const int* nindices, const double* X, double* V);
void lagrangian_ib_4_w8_spread2d_(const double* dx, const double* x_lower, const double* x_upper, const int* depth, const int* indices, const double* Xshift, const int* nindices, const double* X, const double* V, const int* ilower0, const int* iupper0, const int* ilower1, const int* iupper1, const int* nugc0, const int* nugc1, double* u);

/* IB_6 -- lagrangian_interaction3d.f.m4 / lagrangian_interaction2d.f.m4 */
void lagrangian_ib_6_interp3d_(const double* dx, const double* x_lower, const double* x_upper, const int* depth, const int* ilower0, const int* iupper0, const int* ilower1, const int* iupper1, const int* ilower2, const int* iupper2, const int* nugc0, const int* nugc1, const int* nugc2, const double* u, const int* indices, const double* Xshift, const int* nindices, const double* X, double* V);
void lagrangian_ib_6_spread3d_(const double* dx, const double* x_lower, const double* x_upper, const int* depth, const int* indices, const double* Xshift, const int* nindices, const double* X, const double* V, const int* ilower0, const int* iupper0, const int* ilower1, const int* iupper1, const int* ilower2, const int* iupper2, const int* nugc0, const int* nugc1, const int* nugc2, double* u);
void lagrangian_ib_6_interp2d_(const double* dx, const double* x_lower, const double* x_upper, const int* depth, const int* ilower0, const int* iupper0, const int* ilower1, const int* iupper1, const int* nugc0, const int* nugc1, const double* u, const int* indices, const double* Xshift, const int* nindices, const double* X, double* V);
void lagrangian_ib_6_spread2d_(const double* dx, const double* x_lower, const double* x_upper, const int* depth, const int* indices, const double* Xshift, const int* nindices, const double* X, const double* V, const int* ilower0, const int* iupper0, const int* ilower1, const int* iupper1, const int* nugc0, const int* nugc1, double* u);

#ifdef __cplusplus
}
#endif
#endif /* IBTK_LE_FORTRAN_H */
