// clock_probe.hip - diagnostic only (never linked into the product): one
// wave reads the shader-clock counter and the 100 MHz real-time counter
// around a fixed dependent integer loop (-> the shader clock the chip holds
// right now), then walks a dependent chain of loads through lines that are
// cold in every cache (-> the HBM miss latency in ns, which follows the
// memory/fabric clocks). Launched between the product's C2 launches by
// tools/clock_trace.py to see which clock moves during the launch-settling
// transient. Results go to a buffer of their own (vector
// stores); nothing else reads them.
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ void __launch_bounds__(64) clk_probe(uint64_t *out, const uint32_t *chase, uint32_t start, uint32_t hops,
                                                 uint32_t spin)
{
	uint64_t t0 = __builtin_amdgcn_s_memtime();
	uint64_t r0 = __builtin_amdgcn_s_memrealtime();
	uint32_t x = threadIdx.x + 1;
	for (uint32_t i = 0; i < spin; i++)
		x = x * 1664525u + 1013904223u;
	uint64_t t1 = __builtin_amdgcn_s_memtime();
	uint64_t r1 = __builtin_amdgcn_s_memrealtime();
	uint32_t p = start;
	for (uint32_t i = 0; i < hops; i++)
		p = __builtin_nontemporal_load(chase + p);
	uint64_t r2 = __builtin_amdgcn_s_memrealtime();
	if (threadIdx.x == 0) {
		out[0] = t1 - t0;
		out[1] = r1 - r0;
		out[2] = r2 - r1;
		out[3] = (uint64_t)x + p;
	}
}

extern "C" int clk_launch(uint64_t *out, const uint32_t *chase, uint32_t start, uint32_t hops, uint32_t spin,
			  void *stream)
{
	hipLaunchKernelGGL(clk_probe, dim3(1), dim3(64), 0, (hipStream_t)stream, out, chase, start, hops, spin);
	return hipGetLastError() == hipSuccess ? 0 : -1;
}
