// gridrmw.hip — an in-place read-modify-write stream with a chosen grid size (persistent,
// grid-stride), for tools/overlap_probe.py: how much HBM work hides under the next forward when it
// is confined to a few workgroups.
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/gridrmw.hip -o gpurun_variants/libgridrmw.so
#include <hip/hip_runtime.h>
typedef float v4f __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_gridrmw(v4f* __restrict__ p, long n) {
    const long stride = (long)gridDim.x * 256 * 3;
    for (long i = (long)blockIdx.x * 256 * 3 + threadIdx.x; i < n; i += stride) {
        v4f a = p[i];
        v4f b = i + 256 < n ? p[i + 256] : v4f{0, 0, 0, 0};
        v4f c = i + 512 < n ? p[i + 512] : v4f{0, 0, 0, 0};
        p[i] = a * 1.0000001f;
        if (i + 256 < n) p[i + 256] = b * 1.0000001f;
        if (i + 512 < n) p[i + 512] = c * 1.0000001f;
    }
}

extern "C" int gridrmw(float* p, long nfloats, int grid, void* stream) {
    k_gridrmw<<<grid, 256, 0, (hipStream_t)stream>>>(reinterpret_cast<v4f*>(p), nfloats / 4);
    return (int)hipGetLastError();
}
