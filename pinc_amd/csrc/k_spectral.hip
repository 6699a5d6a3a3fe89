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
                                 double Ntot) {
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
	                   f->T[1], f->T[2], (double)f->nReal);
	if (int rc = check_launch("spectral scale")) return rc;
	s = rocfft_execute(f->inv, sp, outp, f->info);
	if (s != rocfft_status_success) return fft_error(s, "fft_poisson: inverse");
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
