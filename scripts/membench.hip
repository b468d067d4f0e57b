// membench.hip -- store-pattern microbenchmark (tooling, not product).
// Writes `rows` rows of 1024 floats with one of several per-lane patterns so
// the cost of the STFT's mirrored dword stores can be compared with plain
// dword / dwordx2 / dwordx4 streaming stores.
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC scripts/membench.hip -o scripts/libmembench.so
#include <hip/hip_runtime.h>

typedef float vf4 __attribute__((ext_vector_type(4)));
typedef float vf2 __attribute__((ext_vector_type(2)));

template <int MODE, bool NT>
__global__ void __launch_bounds__(256) k_wr(float* out, long long rows) {
    const int t = threadIdx.x & 63;
    const long long wave = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
    const long long nw = (long long)gridDim.x * 4;
    const float val = (float)t;
    for (long long row = wave; row < rows; row += nw) {
        float* o = out + row * 1024;
        if constexpr (MODE == 0) {   // dword, lane-contiguous
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                if (NT) __builtin_nontemporal_store(val, o + t + 64 * j);
                else o[t + 64 * j] = val;
            }
        } else if constexpr (MODE == 1) {   // STFT paired-last-pass pattern (k and N-k)
            const int kb0 = t, kb1 = t == 0 ? 128 : 256 - t, kb2 = t + 64, kb3 = 192 - t;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int ks[4] = {kb0 + 256 * r, kb1 + 256 * (3 - r), kb2 + 256 * r, kb3 + 256 * (3 - r)};
#pragma unroll
                for (int s = 0; s < 4; ++s) {
                    if (NT) __builtin_nontemporal_store(val, o + ks[s]);
                    else o[ks[s]] = val;
                }
            }
        } else if constexpr (MODE == 2) {   // dwordx2
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                vf2 v = {val, val};
                vf2* p = reinterpret_cast<vf2*>(o) + t + 64 * j;
                if (NT) __builtin_nontemporal_store(v, p);
                else *p = v;
            }
        } else {   // dwordx4
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                vf4 v = {val, val, val, val};
                vf4* p = reinterpret_cast<vf4*>(o) + t + 64 * j;
                if (NT) __builtin_nontemporal_store(v, p);
                else *p = v;
            }
        }
    }
}

extern "C" int membench_write(float* out, long long rows, int mode, int nt, int blocks, void* stream) {
    hipStream_t s = (hipStream_t)stream;
#define L(M, N) hipLaunchKernelGGL((k_wr<M, N>), dim3(blocks), dim3(256), 0, s, out, rows)
    switch (mode * 2 + (nt ? 1 : 0)) {
        case 0: L(0, false); break; case 1: L(0, true); break;
        case 2: L(1, false); break; case 3: L(1, true); break;
        case 4: L(2, false); break; case 5: L(2, true); break;
        case 6: L(3, false); break; case 7: L(3, true); break;
        default: return -1;
    }
#undef L
    return (int)hipGetLastError();
}
