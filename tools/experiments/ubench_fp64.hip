// FP64 VALU issue microbenchmark (diagnostic, not part of the library): how many cycles a wave64
// v_fma_f64 takes on an MI355X SIMD, and how long a DEPENDENT chain of them stalls a wave, as a
// function of the waves per SIMD and the independent chains per wave. Decides whether the fused
// residual's FP64 phases are bound by issue throughput (more waves do not help) or by dependency
// latency (more independent work per wave / more waves would).
//   hipcc -O3 --offload-arch=gfx950 tools/ubench_fp64.hip -o /tmp/ubench_fp64 && /tmp/ubench_fp64
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define HC(x) do { hipError_t e_ = (x); if(e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while(0)

template <int CH>
__global__ void __launch_bounds__(256) k_chain(double* out, int iters, double a, double b)
{
	extern __shared__ double pad[];             // sized by the launch to set blocks per CU
	double x[CH];
	#pragma unroll
	for(int c = 0; c < CH; c++) x[c] = threadIdx.x * 1e-3 + c;
	for(int i = 0; i < iters; i++) {
		#pragma unroll
		for(int k = 0; k < 8; k++) {
			#pragma unroll
			for(int c = 0; c < CH; c++) x[c] = __builtin_fma(x[c], a, b);
		}
	}
	double s = 0;
	#pragma unroll
	for(int c = 0; c < CH; c++) s += x[c];
	if(s == 12345.678) { pad[0] = s; out[blockIdx.x] = pad[1]; }   // keep the work; never true
}

template <int CH>
int run(int blocksPerCU, double* out)
{
	const int ncu = 256, iters = 4096;
	const size_t lds = (160 * 1024) / blocksPerCU - 1024;
	HC(hipFuncSetAttribute(reinterpret_cast<const void*>(k_chain<CH>), hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds)));
	hipEvent_t e0, e1;
	HC(hipEventCreate(&e0)); HC(hipEventCreate(&e1));
	const int grid = ncu * blocksPerCU;
	for(int w = 0; w < 3; w++) k_chain<CH><<<grid, 256, lds>>>(out, iters, 0.999999, 1e-9);
	HC(hipEventRecord(e0));
	const int reps = 5;
	for(int r = 0; r < reps; r++) k_chain<CH><<<grid, 256, lds>>>(out, iters, 0.999999, 1e-9);
	HC(hipEventRecord(e1));
	HC(hipEventSynchronize(e1));
	float ms = 0;
	HC(hipEventElapsedTime(&ms, e0, e1));
	ms /= reps;
	// per SIMD: blocksPerCU waves (one wave of each 4-wave block per SIMD), each issuing iters*8*CH fmas
	const double fmas_per_simd = static_cast<double>(blocksPerCU) * iters * 8 * CH;
	const double ns_per_fma = ms * 1e6 / fmas_per_simd;
	printf("{\"waves_per_simd\": %d, \"chains_per_wave\": %d, \"ms\": %.4f, \"ns_per_wave_fma_per_simd\": %.4f, "
	       "\"cycles_at_2.4GHz\": %.2f}\n", blocksPerCU, CH, ms, ns_per_fma, ns_per_fma * 2.4);
	return 0;
}

int main()
{
	double* out = nullptr;
	HC(hipMalloc(&out, 1 << 20));
	for(int b : {1, 2, 4}) {
		if(run<1>(b, out) || run<2>(b, out) || run<4>(b, out) || run<8>(b, out)) return 1;
	}
	HC(hipFree(out));
	return 0;
}
