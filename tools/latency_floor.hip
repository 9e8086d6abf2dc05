// Round-trip floors of a synchronous host call on this GPU (tools only): what
// a per-call drop-in search can cost at least, by API shape.
//   hipcc --offload-arch=gfx950 -O2 tools/latency_floor.hip -o /tmp/latency_floor && /tmp/latency_floor
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

__global__ void k_empty(int* p) { if (threadIdx.x == 0 && blockIdx.x == 0 && p) p[0] += 0; }

// reads n words from `in` (host-mapped or device), writes m words to `out`
__global__ void k_touch(const int* __restrict__ in, int n, int* __restrict__ out, int m) {
    int s = 0;
    for (int i = threadIdx.x; i < n; i += blockDim.x) s += in[i];
    __shared__ int red[1024];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int i = threadIdx.x; i < m; i += blockDim.x) out[i] = red[i % blockDim.x] + i;
}

// reads n words of device data, writes m words and then a flag (seq) into
// pinned host memory with system-scope release: the host polls the flag
__global__ void k_touch_flag(const int* __restrict__ in, int n, int* __restrict__ out, int m, int* flag, int seq) {
    int s = 0;
    for (int i = threadIdx.x; i < n; i += blockDim.x) s += in[i];
    __shared__ int red[1024];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int i = threadIdx.x; i < m; i += blockDim.x) out[i] = red[i % blockDim.x] + i;
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        __hip_atomic_store(flag, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// host -> device by a kernel reading the pinned host buffer (16 B a thread)
__global__ void k_pull(const uint4* __restrict__ src, uint4* __restrict__ dst, int n16) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += gridDim.x * blockDim.x) dst[i] = src[i];
}

template <class F> double med_us(F&& f, int reps = 300) {
    for (int i = 0; i < 20; ++i) f();
    std::vector<double> t(reps);
    for (int i = 0; i < reps; ++i) {
        auto a = std::chrono::steady_clock::now();
        f();
        t[i] = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count();
    }
    std::sort(t.begin(), t.end());
    return t[reps / 2];
}

int main() {
    const int NIN = 160 * 1024 / 4, NOUT = 1024;     // ~160 KB in, 4 KB out (a 3000-point projection search)
    int *hin, *hout, *din, *dout;
    CK(hipHostMalloc((void**)&hin, NIN * 4, hipHostMallocDefault));
    CK(hipHostMalloc((void**)&hout, NOUT * 4, hipHostMallocDefault));
    CK(hipMalloc((void**)&din, NIN * 4));
    CK(hipMalloc((void**)&dout, NOUT * 4));
    for (int i = 0; i < NIN; ++i) hin[i] = i;
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    hipError_t err = hipSuccess;
    auto chk = [&](hipError_t e) { if (e != hipSuccess) err = e; };
    std::printf("empty launch + sync (null stream):   %.1f us\n",
                med_us([&] { hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, 0, nullptr); chk(hipStreamSynchronize(0)); }));
    std::printf("empty launch + sync (own stream):    %.1f us\n",
                med_us([&] { hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, st, nullptr); chk(hipStreamSynchronize(st)); }));
    std::printf("H2D 160 KB + sync:                   %.1f us\n",
                med_us([&] { chk(hipMemcpyAsync(din, hin, NIN * 4, hipMemcpyHostToDevice, st)); chk(hipStreamSynchronize(st)); }));
    std::printf("D2H 4 KB + sync:                     %.1f us\n",
                med_us([&] { chk(hipMemcpyAsync(hout, dout, NOUT * 4, hipMemcpyDeviceToHost, st)); chk(hipStreamSynchronize(st)); }));
    auto seq = [&] {
        chk(hipMemcpyAsync(din, hin, NIN * 4, hipMemcpyHostToDevice, st));
        hipLaunchKernelGGL(k_touch, dim3(1), dim3(1024), 0, st, din, NIN, dout, NOUT);
        chk(hipMemcpyAsync(hout, dout, NOUT * 4, hipMemcpyDeviceToHost, st));
        chk(hipStreamSynchronize(st));
    };
    std::printf("H2D + kernel + D2H + sync:           %.1f us\n", med_us(seq));
    auto seq3 = [&] {
        chk(hipMemcpyAsync(din, hin, NIN * 4, hipMemcpyHostToDevice, st));
        hipLaunchKernelGGL(k_touch, dim3(1), dim3(1024), 0, st, din, NIN, dout, NOUT);
        hipLaunchKernelGGL(k_touch, dim3(1), dim3(1024), 0, st, din, NIN, dout, NOUT);
        hipLaunchKernelGGL(k_touch, dim3(1), dim3(1024), 0, st, din, NIN, dout, NOUT);
        chk(hipMemcpyAsync(hout, dout, NOUT * 4, hipMemcpyDeviceToHost, st));
        chk(hipStreamSynchronize(st));
    };
    std::printf("H2D + 3 kernels + D2H + sync:        %.1f us\n", med_us(seq3));
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
    hipMemcpyAsync(din, hin, NIN * 4, hipMemcpyHostToDevice, st);
    hipLaunchKernelGGL(k_touch, dim3(1), dim3(1024), 0, st, din, NIN, dout, NOUT);
    hipMemcpyAsync(hout, dout, NOUT * 4, hipMemcpyDeviceToHost, st);
    CK(hipStreamEndCapture(st, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    std::printf("graph(H2D + kernel + D2H) + sync:    %.1f us\n",
                med_us([&] { chk(hipGraphLaunch(ge, st)); chk(hipStreamSynchronize(st)); }));
    // the same graph with its three nodes' parameters set again before every
    // launch (what a per-call graph of a host API with varying sizes pays)
    {
        size_t nn = 0;
        CK(hipGraphGetNodes(g, nullptr, &nn));
        std::vector<hipGraphNode_t> nodes(nn);
        CK(hipGraphGetNodes(g, nodes.data(), &nn));
        hipGraphNode_t kn = nullptr, h2d = nullptr, d2h = nullptr;
        for (auto nd : nodes) {
            hipGraphNodeType t;
            CK(hipGraphNodeGetType(nd, &t));
            if (t == hipGraphNodeTypeKernel) kn = nd;
            else if (t == hipGraphNodeTypeMemcpy) (h2d ? d2h : h2d) = nd;
        }
        hipKernelNodeParams kp{};
        CK(hipGraphKernelNodeGetParams(kn, &kp));
        int nin = NIN, nout = NOUT;
        void* args[4] = {&din, &nin, &dout, &nout};
        kp.kernelParams = args;
        std::printf("graph + per-launch node updates:     %.1f us\n", med_us([&] {
            chk(hipGraphExecMemcpyNodeSetParams1D(ge, h2d, din, hin, NIN * 4, hipMemcpyHostToDevice));
            chk(hipGraphExecKernelNodeSetParams(ge, kn, &kp));
            chk(hipGraphExecMemcpyNodeSetParams1D(ge, d2h, hout, dout, NOUT * 4, hipMemcpyDeviceToHost));
            chk(hipGraphLaunch(ge, st));
            chk(hipStreamSynchronize(st));
        }));
    }
    // zero-copy: the kernel reads the pinned host inputs and writes the pinned host outputs
    int *hin_d, *hout_d;
    CK(hipHostGetDevicePointer((void**)&hin_d, hin, 0));
    CK(hipHostGetDevicePointer((void**)&hout_d, hout, 0));
    std::printf("zero-copy kernel (1 block) + sync:   %.1f us\n",
                med_us([&] { hipLaunchKernelGGL(k_touch, dim3(1), dim3(1024), 0, st, hin_d, NIN, hout_d, NOUT); chk(hipStreamSynchronize(st)); }));
    {
        int* hflag;
        CK(hipHostMalloc((void**)&hflag, 64, hipHostMallocDefault));
        int *hflag_d, *hout_d2;
        CK(hipHostGetDevicePointer((void**)&hflag_d, hflag, 0));
        CK(hipHostGetDevicePointer((void**)&hout_d2, hout, 0));
        volatile int* vf = hflag;
        int seq = 0;
        *vf = 0;
        std::printf("kernel + host poll (no sync):        %.1f us\n", med_us([&] {
            ++seq;
            hipLaunchKernelGGL(k_touch_flag, dim3(1), dim3(1024), 0, st, din, NIN, hout_d2, NOUT, hflag_d, seq);
            while (*vf != seq) {}
        }));
        std::printf("H2D + kernel + host poll:            %.1f us\n", med_us([&] {
            ++seq;
            chk(hipMemcpyAsync(din, hin, NIN * 4, hipMemcpyHostToDevice, st));
            hipLaunchKernelGGL(k_touch_flag, dim3(1), dim3(1024), 0, st, din, NIN, hout_d2, NOUT, hflag_d, seq);
            while (*vf != seq) {}
        }));
        std::printf("H2D + kernel + host poll + sync:     %.1f us\n", med_us([&] {
            ++seq;
            chk(hipMemcpyAsync(din, hin, NIN * 4, hipMemcpyHostToDevice, st));
            hipLaunchKernelGGL(k_touch_flag, dim3(1), dim3(1024), 0, st, din, NIN, hout_d2, NOUT, hflag_d, seq);
            while (*vf != seq) {}
            chk(hipStreamSynchronize(st));
        }));
        int* hin_d2;
        CK(hipHostGetDevicePointer((void**)&hin_d2, hin, 0));
        for (int nb : {16, 64, 160}) {
            std::printf("pull kernel(%3d blk) + kernel + poll: %.1f us\n", nb, med_us([&] {
                ++seq;
                hipLaunchKernelGGL(k_pull, dim3(nb), dim3(256), 0, st, (const uint4*)hin_d2, (uint4*)din, NIN / 4);
                hipLaunchKernelGGL(k_touch_flag, dim3(1), dim3(1024), 0, st, din, NIN, hout_d2, NOUT, hflag_d, seq);
                while (*vf != seq) {}
            }));
        }
        std::printf("pull + kernel + poll + D2H-free sync: %.1f us\n", med_us([&] {
            ++seq;
            hipLaunchKernelGGL(k_pull, dim3(64), dim3(256), 0, st, (const uint4*)hin_d2, (uint4*)din, NIN / 4);
            hipLaunchKernelGGL(k_touch_flag, dim3(1), dim3(1024), 0, st, din, NIN, hout_d2, NOUT, hflag_d, seq);
            chk(hipStreamSynchronize(st));
        }));
        std::printf("H2D + kernel + sync (zero-copy out): %.1f us\n", med_us([&] {
            ++seq;
            chk(hipMemcpyAsync(din, hin, NIN * 4, hipMemcpyHostToDevice, st));
            hipLaunchKernelGGL(k_touch_flag, dim3(1), dim3(1024), 0, st, din, NIN, hout_d2, NOUT, hflag_d, seq);
            chk(hipStreamSynchronize(st));
        }));
    }
    std::printf("kernel alone on device data + sync:  %.1f us\n",
                med_us([&] { hipLaunchKernelGGL(k_touch, dim3(1), dim3(1024), 0, st, din, NIN, dout, NOUT); chk(hipStreamSynchronize(st)); }));
    std::printf("status: %s\n", hipGetErrorString(err));
    return 0;
}
