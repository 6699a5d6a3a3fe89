// k_spectral.hip -- spectral Poisson solve (sSolve, spectral.c:92-115) on
// rocFFT for MI355X (gfx950).
//
// The reference solves -lap(phi) = rho in 1-D with FFTW (spectral.c:14-52):
// r2c of rho, spectrum[0] = 0, spectrum[n] *= (N/(2 pi n))^2 / N, c2r.  This
// is the same operator on the whole periodic domain of 1, 2 or 3 dimensions
// (the 1-D factor is reproduced expression by expression; in N-D the factor
// is 1/|k|^2/N with k_d = 2 pi n_d/N_d, n_d the signed frequency):
//
//   rho (global, [Tz][Ty][Tx] x fastest) --r2c--> spec [Tz][Ty][Tx/2+1]
//   spec *= factor(k) in k_spectral_scale (DC -> 0)
//   spec --c2r--> phi (global)
//
// Plans are made once per grid shape (sAlloc); rocFFT's work buffer and the
// spectrum live in HBM next to the grids.  rho is copied into a private
// real buffer first, so no transform can touch the caller's rho.
#include "common.h"
#include <rocfft/rocfft.h>
#include <math.h>

using namespace pinc;

struct pinc_fft_s {
	int nd;
	int T[3];
	long nReal, nSpec;
	rocfft_plan fwd, inv;
	rocfft_execution_info info;
	void *work;
	double *rin;      // private copy of rho
	double2 *spec;    // half spectrum
	int discrete;     // k-space factor of the discrete Laplacian (pinc_hip_fft_set_symbol)
};

namespace {

bool g_rocfft_ready = false;
int g_rocfft_plans = 0;  // live plans (pinc_hip_fft_create / _destroy)

int fft_error(rocfft_status s, const char *where) {
	if (s == rocfft_status_success) return 0;
	return set_error(hipErrorUnknown, where);
}

// spec[i] *= factor(i), spectral.c:29-37 (1-D) generalised to N-D
__global__ void k_spectral_scale(double2 *__restrict__ spec, long n, int nd, int Tx, int Ty, int Tz,
                                 double Ntot, int discrete) {
	for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
		int Mx = Tx / 2 + 1;
		long r = i;
		int ix = (int)(r % Mx);
		r /= Mx;
		int iy = nd > 1 ? (int)(r % Ty) : 0;
		r = nd > 1 ? r / Ty : r;
		int iz = nd > 2 ? (int)r : 0;
		double f;
		if (i == 0) {
			f = 0.0;  // charge neutrality (spectral.c:103-104)
		} else if (discrete) {
			// -(sum of the 2 nd neighbours - 2 nd phi) = rho, mode by mode
			int ny = iy <= Ty / 2 ? iy : iy - Ty;
			int nz = iz <= Tz / 2 ? iz : iz - Tz;
			double s = 2.0 - 2.0 * cos(2 * M_PI * ix / Tx);
			if (nd > 1) s += 2.0 - 2.0 * cos(2 * M_PI * ny / Ty);
			if (nd > 2) s += 2.0 - 2.0 * cos(2 * M_PI * nz / Tz);
			f = 1.0 / s / Ntot;
		} else if (nd == 1) {
			f = Tx / (2 * M_PI * ix);  // size/(2*M_PI*n), squared, /size
			f *= f;
			f /= Tx;
		} else {
			int ny = iy <= Ty / 2 ? iy : iy - Ty;
			int nz = iz <= Tz / 2 ? iz : iz - Tz;
			double kx = 2 * M_PI * ix / Tx, ky = 2 * M_PI * ny / Ty, kz = nd > 2 ? 2 * M_PI * nz / Tz : 0.0;
			f = 1.0 / (kx * kx + ky * ky + kz * kz);
			f /= Ntot;
		}
		double2 v = spec[i];
		v.x *= f;
		v.y *= f;
		spec[i] = v;
	}
}

}  // namespace

extern "C" int pinc_hip_fft_create(pinc_fft_t **out, int nd, const int *T, void *stream) {
	(void)stream;
	*out = nullptr;
	if (nd < 1 || nd > 3) return set_error(hipErrorInvalidValue, "fft_create: nDims");
	if (!g_rocfft_ready) {
		if (int rc = fft_error(rocfft_setup(), "rocfft_setup")) return rc;
		g_rocfft_ready = true;
	}
	pinc_fft_t *f = (pinc_fft_t *)calloc(1, sizeof(pinc_fft_t));
	g_rocfft_plans++;
	f->nd = nd;
	f->nReal = 1;
	for (int d = 0; d < 3; d++) {
		f->T[d] = d < nd ? T[d] : 1;
		f->nReal *= f->T[d];
	}
	if (f->T[0] % 2) {
		free(f);
		return set_error(hipErrorInvalidValue, "fft_create: x size must be even");
	}
	f->nSpec = f->nReal / f->T[0] * (f->T[0] / 2 + 1);
	size_t len[3] = {(size_t)f->T[0], (size_t)f->T[1], (size_t)f->T[2]};  // fastest first
	rocfft_status s = rocfft_plan_create(&f->fwd, rocfft_placement_notinplace, rocfft_transform_type_real_forward,
	                                     rocfft_precision_double, nd, len, 1, nullptr);
	if (s == rocfft_status_success)
		s = rocfft_plan_create(&f->inv, rocfft_placement_notinplace, rocfft_transform_type_real_inverse,
		                       rocfft_precision_double, nd, len, 1, nullptr);
	size_t w1 = 0, w2 = 0;
	if (s == rocfft_status_success) s = rocfft_plan_get_work_buffer_size(f->fwd, &w1);
	if (s == rocfft_status_success) s = rocfft_plan_get_work_buffer_size(f->inv, &w2);
	if (s == rocfft_status_success) s = rocfft_execution_info_create(&f->info);
	if (s != rocfft_status_success) {
		pinc_hip_fft_destroy(f);
		return fft_error(s, "fft_create: plan");
	}
	size_t w = w1 > w2 ? w1 : w2;
	hipError_t e = hipSuccess;
	if (w) e = hipMalloc(&f->work, w);
	if (e == hipSuccess) e = hipMalloc((void **)&f->rin, f->nReal * sizeof(double));
	if (e == hipSuccess) e = hipMalloc((void **)&f->spec, f->nSpec * sizeof(double2));
	if (e != hipSuccess) {
		pinc_hip_fft_destroy(f);
		return set_error(e, "fft_create: buffers");
	}
	if (w) {
		s = rocfft_execution_info_set_work_buffer(f->info, f->work, w);
		if (s != rocfft_status_success) {
			pinc_hip_fft_destroy(f);
			return fft_error(s, "fft_create: work buffer");
		}
	}
	*out = f;
	return 0;
}

extern "C" int pinc_hip_fft_poisson(pinc_fft_t *f, const double *rho, double *phi, void *stream) {
	hipStream_t st = (hipStream_t)stream;
	hipError_t e = hipMemcpyAsync(f->rin, rho, f->nReal * sizeof(double), hipMemcpyDeviceToDevice, st);
	if (e != hipSuccess) return set_error(e, "fft_poisson: copy");
	rocfft_status s = rocfft_execution_info_set_stream(f->info, st);
	if (s != rocfft_status_success) return fft_error(s, "fft_poisson: stream");
	void *in[1] = {f->rin}, *sp[1] = {f->spec}, *outp[1] = {phi};
	s = rocfft_execute(f->fwd, in, sp, f->info);
	if (s != rocfft_status_success) return fft_error(s, "fft_poisson: forward");
	long nb = (f->nSpec + 255) / 256;
	if (nb > 8192) nb = 8192;
	hipLaunchKernelGGL(k_spectral_scale, dim3((unsigned)nb), dim3(256), 0, st, f->spec, f->nSpec, f->nd, f->T[0],
	                   f->T[1], f->T[2], (double)f->nReal, f->discrete);
	if (int rc = check_launch("spectral scale")) return rc;
	s = rocfft_execute(f->inv, sp, outp, f->info);
	if (s != rocfft_status_success) return fft_error(s, "fft_poisson: inverse");
	return 0;
}

extern "C" int pinc_hip_fft_set_symbol(pinc_fft_t *f, int discrete) {
	if (!f) return set_error(hipErrorInvalidValue, "fft_set_symbol: no plan");
	f->discrete = discrete != 0;
	return 0;
}

extern "C" void pinc_hip_fft_destroy(pinc_fft_t *f) {
	if (!f) return;
	if (f->fwd) rocfft_plan_destroy(f->fwd);
	if (f->inv) rocfft_plan_destroy(f->inv);
	if (f->info) rocfft_execution_info_destroy(f->info);
	if (f->work) (void)hipFree(f->work);
	if (f->rin) (void)hipFree(f->rin);
	if (f->spec) (void)hipFree(f->spec);
	free(f);
	// rocfft_setup is paired with rocfft_cleanup once the last plan is gone,
	// so rocFFT's state is released while the HIP runtime is still up
	// instead of by static destructors after it
	if (--g_rocfft_plans == 0 && g_rocfft_ready) {
		(void)rocfft_cleanup();
		g_rocfft_ready = false;
	}
}

// --------------------------------------------------- slab-distributed 3-D ---
// the 3-D solve over P z-slabs without gathering rho.  Rank
// r holds planes [r nloc, (r+1) nloc).
//   1. batched 2-D r2c over its planes:        A [zl][y][kx]   (kx < Mx)
//   2. pack by destination ky block (Ty/P rows): S [q][zl][yl][kx]
//   3. all-to-all (host: pinc_comm_exchange):  B [p][zl][yl][kx] = [z][yl][kx],
//      rank r now holds ky in [r Tyl, (r+1) Tyl) for every z
//   4. 1-D c2c along z (stride Tyl Mx), the factor of k_spectral_scale at
//      the global (kx, ky, kz), inverse c2c along z
//   5. all-to-all back (B's z blocks to their slabs) into S, unpack into A,
//      batched 2-D c2r into the phi slab.
// The same operator as the single-plan solve; the transforms are split, so
// results agree to FFT round-off, not bit for bit.
struct pinc_fft_slab_s {
	int T[3], nloc, P, rank, Tyl, Mx;
	int discrete;     // the 7-point symbol (pinc_hip_fft_slab_set_symbol)
	long nBlock;      // complex values per (rank pair) block: nloc * Tyl * Mx
	rocfft_plan fwd2, inv2, zfwd, zinv;
	rocfft_execution_info info;
	void *work;
	double *rin;
	double2 *A, *S, *B;
};

namespace {

__global__ void k_slab_pack(const double2 *__restrict__ A, double2 *__restrict__ S, int nloc, int Ty, int Tyl, int Mx,
                            int P) {
	// S [q][zl][yl][kx] <- A [zl][q Tyl + yl][kx]
	const long n = (long)P * nloc * Tyl * Mx;
	for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
		const int kx = (int)(i % Mx);
		long r = i / Mx;
		const int yl = (int)(r % Tyl);
		r /= Tyl;
		const int zl = (int)(r % nloc);
		const int q = (int)(r / nloc);
		S[i] = A[((long)zl * Ty + (long)q * Tyl + yl) * Mx + kx];
	}
}

__global__ void k_slab_unpack(const double2 *__restrict__ S, double2 *__restrict__ A, int nloc, int Ty, int Tyl,
                              int Mx, int P) {
	// A [zl][p Tyl + yl][kx] <- S [p][zl][yl][kx]
	const long n = (long)P * nloc * Tyl * Mx;
	for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
		const int kx = (int)(i % Mx);
		long r = i / Mx;
		const int yl = (int)(r % Tyl);
		r /= Tyl;
		const int zl = (int)(r % nloc);
		const int p = (int)(r / nloc);
		A[((long)zl * Ty + (long)p * Tyl + yl) * Mx + kx] = S[i];
	}
}

// B [z][yl][kx] *= factor at (kx, ky = y0 + yl, kz = z): k_spectral_scale's 3-D
// branches (continuous or discrete symbol)
__global__ void k_slab_scale(double2 *__restrict__ B, int Tx, int Ty, int Tz, int Tyl, int y0, double Ntot,
                             int discrete) {
	const int Mx = Tx / 2 + 1;
	const long n = (long)Tz * Tyl * Mx;
	for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
		const int ix = (int)(i % Mx);
		long r = i / Mx;
		const int iy = y0 + (int)(r % Tyl);
		const int iz = (int)(r / Tyl);
		double f;
		if (ix == 0 && iy == 0 && iz == 0) {
			f = 0.0;  // charge neutrality (spectral.c:103-104)
		} else {
			const int ny = iy <= Ty / 2 ? iy : iy - Ty;
			const int nz = iz <= Tz / 2 ? iz : iz - Tz;
			if (discrete) {
				const double s = (2.0 - 2.0 * cos(2 * M_PI * ix / Tx)) + (2.0 - 2.0 * cos(2 * M_PI * ny / Ty)) +
				                 (2.0 - 2.0 * cos(2 * M_PI * nz / Tz));
				f = 1.0 / s / Ntot;
			} else {
				const double kx = 2 * M_PI * ix / Tx, ky = 2 * M_PI * ny / Ty, kz = 2 * M_PI * nz / Tz;
				f = 1.0 / (kx * kx + ky * ky + kz * kz);
				f /= Ntot;
			}
		}
		double2 v = B[i];
		v.x *= f;
		v.y *= f;
		B[i] = v;
	}
}

unsigned slab_blocks(long n) {
	long b = (n + 255) / 256;
	return (unsigned)(b > 8192 ? 8192 : (b < 1 ? 1 : b));
}

}  // namespace

extern "C" void pinc_hip_fft_slab_destroy(pinc_fft_slab_t *f) {
	if (!f) return;
	if (f->fwd2) rocfft_plan_destroy(f->fwd2);
	if (f->inv2) rocfft_plan_destroy(f->inv2);
	if (f->zfwd) rocfft_plan_destroy(f->zfwd);
	if (f->zinv) rocfft_plan_destroy(f->zinv);
	if (f->info) rocfft_execution_info_destroy(f->info);
	(void)hipFree(f->work);
	(void)hipFree(f->rin);
	(void)hipFree(f->A);
	(void)hipFree(f->S);
	(void)hipFree(f->B);
	free(f);
	if (--g_rocfft_plans == 0 && g_rocfft_ready) {
		(void)rocfft_cleanup();
		g_rocfft_ready = false;
	}
}

extern "C" int pinc_hip_fft_slab_create(pinc_fft_slab_t **out, const int *T, int nloc, int nranks, int rank,
                                        void *stream) {
	(void)stream;
	*out = nullptr;
	if (T[0] % 2 || nranks < 1 || T[1] % nranks || T[2] != nloc * nranks || rank < 0 || rank >= nranks)
		return set_error(hipErrorInvalidValue, "fft_slab_create: even Tx, Ty divisible by the ranks, Tz = nloc ranks");
	if (!g_rocfft_ready) {
		if (int rc = fft_error(rocfft_setup(), "rocfft_setup")) return rc;
		g_rocfft_ready = true;
	}
	pinc_fft_slab_t *f = (pinc_fft_slab_t *)calloc(1, sizeof(pinc_fft_slab_t));
	g_rocfft_plans++;
	for (int d = 0; d < 3; d++) f->T[d] = T[d];
	f->nloc = nloc;
	f->P = nranks;
	f->rank = rank;
	f->Tyl = T[1] / nranks;
	f->Mx = T[0] / 2 + 1;
	f->nBlock = (long)nloc * f->Tyl * f->Mx;
	const long nSpec = f->nBlock * nranks;  // = nloc Ty Mx = Tz Tyl Mx
	size_t len2[2] = {(size_t)T[0], (size_t)T[1]};
	rocfft_status s = rocfft_plan_create(&f->fwd2, rocfft_placement_notinplace, rocfft_transform_type_real_forward,
	                                     rocfft_precision_double, 2, len2, (size_t)nloc, nullptr);
	if (s == rocfft_status_success)
		s = rocfft_plan_create(&f->inv2, rocfft_placement_notinplace, rocfft_transform_type_real_inverse,
		                       rocfft_precision_double, 2, len2, (size_t)nloc, nullptr);
	// along z: length Tz, stride Tyl Mx, one transform per (yl, kx)
	rocfft_plan_description desc = nullptr;
	if (s == rocfft_status_success) s = rocfft_plan_description_create(&desc);
	size_t lenz[1] = {(size_t)T[2]}, strz[1] = {(size_t)f->Tyl * f->Mx};
	if (s == rocfft_status_success)
		s = rocfft_plan_description_set_data_layout(desc, rocfft_array_type_complex_interleaved,
		                                            rocfft_array_type_complex_interleaved, nullptr, nullptr, 1, strz, 1, 1,
		                                            strz, 1);
	if (s == rocfft_status_success)
		s = rocfft_plan_create(&f->zfwd, rocfft_placement_inplace, rocfft_transform_type_complex_forward,
		                       rocfft_precision_double, 1, lenz, strz[0], desc);
	if (s == rocfft_status_success)
		s = rocfft_plan_create(&f->zinv, rocfft_placement_inplace, rocfft_transform_type_complex_inverse,
		                       rocfft_precision_double, 1, lenz, strz[0], desc);
	if (desc) rocfft_plan_description_destroy(desc);
	size_t w = 0;
	rocfft_plan plans[4] = {f->fwd2, f->inv2, f->zfwd, f->zinv};
	for (int k = 0; k < 4 && s == rocfft_status_success; k++) {
		size_t wk = 0;
		s = rocfft_plan_get_work_buffer_size(plans[k], &wk);
		if (wk > w) w = wk;
	}
	if (s == rocfft_status_success) s = rocfft_execution_info_create(&f->info);
	if (s != rocfft_status_success) {
		pinc_hip_fft_slab_destroy(f);
		return fft_error(s, "fft_slab_create: plans");
	}
	hipError_t e = hipSuccess;
	if (w) e = hipMalloc(&f->work, w);
	if (e == hipSuccess) e = hipMalloc((void **)&f->rin, (size_t)nloc * T[0] * T[1] * sizeof(double));
	if (e == hipSuccess) e = hipMalloc((void **)&f->A, nSpec * sizeof(double2));
	if (e == hipSuccess) e = hipMalloc((void **)&f->S, nSpec * sizeof(double2));
	if (e == hipSuccess) e = hipMalloc((void **)&f->B, nSpec * sizeof(double2));
	if (e != hipSuccess) {
		pinc_hip_fft_slab_destroy(f);
		return set_error(e, "fft_slab_create: buffers");
	}
	if (w && (s = rocfft_execution_info_set_work_buffer(f->info, f->work, w)) != rocfft_status_success) {
		pinc_hip_fft_slab_destroy(f);
		return fft_error(s, "fft_slab_create: work buffer");
	}
	*out = f;
	return 0;
}

extern "C" int pinc_hip_fft_slab_set_symbol(pinc_fft_slab_t *f, int discrete) {
	if (!f) return set_error(hipErrorInvalidValue, "fft_slab_set_symbol: no plan");
	f->discrete = discrete != 0;
	return 0;
}

extern "C" int pinc_hip_fft_slab_buffers(pinc_fft_slab_t *f, void **S, void **B, long *blockBytes) {
	*S = f->S;
	*B = f->B;
	*blockBytes = f->nBlock * (long)sizeof(double2);
	return 0;
}

extern "C" int pinc_hip_fft_slab_forward(pinc_fft_slab_t *f, const double *rhoSlab, void *stream) {
	hipStream_t st = (hipStream_t)stream;
	hipError_t e = hipMemcpyAsync(f->rin, rhoSlab, (size_t)f->nloc * f->T[0] * f->T[1] * sizeof(double),
	                              hipMemcpyDeviceToDevice, st);
	if (e != hipSuccess) return set_error(e, "fft_slab_forward: copy");
	rocfft_status s = rocfft_execution_info_set_stream(f->info, st);
	void *in[1] = {f->rin}, *out[1] = {f->A};
	if (s == rocfft_status_success) s = rocfft_execute(f->fwd2, in, out, f->info);
	if (s != rocfft_status_success) return fft_error(s, "fft_slab_forward: r2c");
	hipLaunchKernelGGL(k_slab_pack, dim3(slab_blocks(f->nBlock * f->P)), dim3(256), 0, st, f->A, f->S, f->nloc,
	                   f->T[1], f->Tyl, f->Mx, f->P);
	return check_launch("fft_slab_forward: pack");
}

extern "C" int pinc_hip_fft_slab_kspace(pinc_fft_slab_t *f, void *stream) {
	hipStream_t st = (hipStream_t)stream;
	rocfft_status s = rocfft_execution_info_set_stream(f->info, st);
	void *io[1] = {f->B};
	if (s == rocfft_status_success) s = rocfft_execute(f->zfwd, io, nullptr, f->info);
	if (s != rocfft_status_success) return fft_error(s, "fft_slab_kspace: z forward");
	hipLaunchKernelGGL(k_slab_scale, dim3(slab_blocks(f->nBlock * f->P)), dim3(256), 0, st, f->B, f->T[0], f->T[1],
	                   f->T[2], f->Tyl, f->rank * f->Tyl, (double)f->T[0] * f->T[1] * f->T[2], f->discrete);
	if (int rc = check_launch("fft_slab_kspace: scale")) return rc;
	s = rocfft_execute(f->zinv, io, nullptr, f->info);
	if (s != rocfft_status_success) return fft_error(s, "fft_slab_kspace: z inverse");
	return 0;
}

extern "C" int pinc_hip_fft_slab_backward(pinc_fft_slab_t *f, double *phiSlab, void *stream) {
	hipStream_t st = (hipStream_t)stream;
	hipLaunchKernelGGL(k_slab_unpack, dim3(slab_blocks(f->nBlock * f->P)), dim3(256), 0, st, f->S, f->A, f->nloc,
	                   f->T[1], f->Tyl, f->Mx, f->P);
	if (int rc = check_launch("fft_slab_backward: unpack")) return rc;
	rocfft_status s = rocfft_execution_info_set_stream(f->info, st);
	void *in[1] = {f->A}, *out[1] = {phiSlab};
	if (s == rocfft_status_success) s = rocfft_execute(f->inv2, in, out, f->info);
	if (s != rocfft_status_success) return fft_error(s, "fft_slab_backward: c2r");
	return 0;
}
