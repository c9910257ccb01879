// Host enqueue cost of one partitioned rank's residual step, on one GPU.
// The RCCL rank step (ctx.hpp residual_fused_overlapped) enqueues: event record + stream wait, the pack,
// ncclGroupStart, one ncclSend/ncclRecv pair per neighbour, ncclGroupEnd, the layer-1 ghost gradients,
// the interior and the border fused launches, event record + stream wait. RCCL refuses two ranks on one
// device, so the pairs here go to the rank itself over a 1-rank communicator with the rank's own
// per-neighbour row counts; the residual launches are the library's own (fvhip_compute_residual_device
// with FVHIP_RES_HALO_READY: k_grad_ghost + the fused kernel), the pack a device copy of the send rows.
// Built by tools/enqueue_probe.py (hipcc, -lrccl); driven from Python through ctypes.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <chrono>
#include <cstdio>
#include "../../include/fvhip.h"

#define HCK(x) do { hipError_t e_ = (x); if(e_ != hipSuccess) { std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while(0)
#define NCK(x) do { ncclResult_t e_ = (x); if(e_ != ncclSuccess) { std::fprintf(stderr, "%s: %s\n", #x, ncclGetErrorString(e_)); return 2; } } while(0)

static double now_us() {
	return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

/// out[0..5]: full step host enqueue us/step, full step wall us/step (enqueue + drain), residual-only
/// host us/step, residual-only wall us/step, exchange-only host us/step, exchange-only wall us/step
extern "C" int enq_probe(fvhip_handle h, const double* du, double* dr, double* ddt, int nnbr, const int* counts,
                         double* sendbuf, double* recvbuf, int iters, double* out)
{
	hipStream_t st = static_cast<hipStream_t>(fvhip_stream(h));
	if(!st) { std::fprintf(stderr, "no stream\n"); return 3; }
	ncclUniqueId id;
	NCK(ncclGetUniqueId(&id));
	ncclComm_t comm;
	NCK(ncclCommInitRank(&comm, 1, id, 0));
	hipStream_t cs;
	HCK(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
	hipEvent_t ev_u, ev_halo;
	HCK(hipEventCreateWithFlags(&ev_u, hipEventDisableTiming));
	HCK(hipEventCreateWithFlags(&ev_halo, hipEventDisableTiming));
	long long total = 0;
	for(int k = 0; k < nnbr; k++) total += counts[k];
	auto exchange = [&]() -> int {
		HCK(hipEventRecord(ev_u, st));
		HCK(hipStreamWaitEvent(cs, ev_u, 0));
		HCK(hipMemcpyAsync(sendbuf, recvbuf, sizeof(double)*4*total, hipMemcpyDeviceToDevice, cs));   // the pack
		NCK(ncclGroupStart());
		long long off = 0;
		for(int k = 0; k < nnbr; k++) {
			NCK(ncclSend(sendbuf + 4*off, 4*static_cast<size_t>(counts[k]), ncclDouble, 0, comm, cs));
			NCK(ncclRecv(recvbuf + 4*off, 4*static_cast<size_t>(counts[k]), ncclDouble, 0, comm, cs));
			off += counts[k];
		}
		NCK(ncclGroupEnd());
		return 0;
	};
	auto finish = [&]() -> int {
		HCK(hipEventRecord(ev_halo, cs));
		HCK(hipStreamWaitEvent(st, ev_halo, 0));
		return 0;
	};
	auto residual = [&]() -> int {
		if(fvhip_compute_residual_device(h, du, dr, 1, ddt, FVHIP_RES_OVERWRITE | FVHIP_RES_HALO_READY)) {
			std::fprintf(stderr, "%s\n", fvhip_last_error()); return 4;
		}
		return 0;
	};
	for(int mode = 0; mode < 3; mode++) {
		for(int w = 0; w < 20; w++) {                  // warm-up (RCCL connection set-up, code objects)
			if(mode != 1 && exchange()) return 5;
			if(mode != 2 && residual()) return 5;
			if(mode != 1 && finish()) return 5;
		}
		HCK(hipDeviceSynchronize());
		const double t0 = now_us();
		for(int i = 0; i < iters; i++) {
			if(mode != 1 && exchange()) return 5;
			if(mode != 2 && residual()) return 5;
			if(mode != 1 && finish()) return 5;
		}
		const double t1 = now_us();
		HCK(hipDeviceSynchronize());
		const double t2 = now_us();
		out[2*mode] = (t1 - t0)/iters;
		out[2*mode+1] = (t2 - t0)/iters;
	}
	HCK(hipEventDestroy(ev_u));
	HCK(hipEventDestroy(ev_halo));
	HCK(hipStreamDestroy(cs));
	NCK(ncclCommDestroy(comm));
	return 0;
}
