// Access-pattern probe for the SSCS vote (tuning experiment, not product code).
// 20M records in 256-B payload slots (160 B quals + 80 B nibbles, the L = 150 layout), grouped
// into families of 1 + Poisson(3)-like sizes made of consecutive records.  Times:
//   stream   : every slot read once, 16 B per lane, in address order
//   gather   : lane = (family, 16-position chunk), per member one 16-B + one 8-B load (vote pattern)
//   gather_p : the same, families visited in a shuffled order (vote-slot order stand-in)
//   lds      : block loads its contiguous record range into LDS (16 B per lane, coalesced), then the
//              vote pattern reads LDS
// Build: hipcc --offload-arch=gfx950 -O3 -o probe_gather probe_gather.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <random>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

constexpr int SLOT = 256, CH = 10, FPW = 6;

__global__ void k_stream(const uint4* __restrict__ p, int64_t n16, uint32_t* out) {
    uint32_t acc = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (int64_t)gridDim.x * blockDim.x) {
        const uint4 v = p[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// fam_beg[f], fam_cnt[f] in records; order[] = family visit order
__global__ void k_gather(const uint8_t* __restrict__ pay, const int32_t* __restrict__ order, const int32_t* __restrict__ fam_beg,
                         const int32_t* __restrict__ fam_cnt, int64_t nf, uint32_t* out) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int g = lane / CH, c = lane - g * CH;
    const int64_t fi = wave * FPW + g;
    uint32_t acc = 0;
    if (g < FPW && fi < nf) {
        const int32_t f = order[fi];
        const int32_t b = fam_beg[f], n = fam_cnt[f];
        for (int k0 = 0; k0 < n; k0 += 4) {
            uint4 q[4]; uint2 s[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                q[u] = make_uint4(0, 0, 0, 0); s[u] = make_uint2(0, 0);
                if (k0 + u < n) {
                    const uint8_t* r = pay + (int64_t)(b + k0 + u) * SLOT;
                    q[u] = *reinterpret_cast<const uint4*>(r + 16 * c);
                    s[u] = *reinterpret_cast<const uint2*>(r + 160 + 8 * c);
                }
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) acc += q[u].x ^ q[u].y ^ q[u].z ^ q[u].w ^ s[u].x ^ s[u].y;
        }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// block = 256 consecutive records (64 KB) staged in LDS, then families starting in the block are
// voted from LDS (families cut at the block edge are simply read from global here)
__global__ __launch_bounds__(256) void k_lds(const uint8_t* __restrict__ pay, const int32_t* __restrict__ first_fam,
                                             const int32_t* __restrict__ fam_beg, const int32_t* __restrict__ fam_cnt,
                                             int64_t nrec, int64_t nf, uint32_t* out) {
    extern __shared__ uint4 lds[];
    const int64_t r0 = (int64_t)blockIdx.x * 256;
    const int64_t r1 = min(r0 + 256, nrec);
    const uint4* src = reinterpret_cast<const uint4*>(pay + r0 * SLOT);
    const int n16 = (int)((r1 - r0) * SLOT / 16);
    for (int i = threadIdx.x; i < n16; i += 256) lds[i] = src[i];
    __syncthreads();
    const int f0 = first_fam[blockIdx.x], f1 = first_fam[blockIdx.x + 1];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int g = lane / CH, c = lane - g * CH;
    uint32_t acc = 0;
    for (int fb = f0 + wv * FPW; fb < f1; fb += 4 * FPW) {
        const int f = fb + g;
        if (g >= FPW || f >= f1) continue;
        const int32_t b = fam_beg[f], n = fam_cnt[f];
        for (int k = 0; k < n; ++k) {
            const int64_t r = b + k;
            uint4 q; uint2 s;
            if (r < r1) {
                const uint8_t* lr = reinterpret_cast<const uint8_t*>(lds) + (r - r0) * SLOT;
                q = *reinterpret_cast<const uint4*>(lr + 16 * c);
                s = *reinterpret_cast<const uint2*>(lr + 160 + 8 * c);
            } else {
                const uint8_t* gr = pay + r * SLOT;
                q = *reinterpret_cast<const uint4*>(gr + 16 * c);
                s = *reinterpret_cast<const uint2*>(gr + 160 + 8 * c);
            }
            acc += q.x ^ q.y ^ q.z ^ q.w ^ s.x ^ s.y;
        }
    }
    if (acc == 0x12345678u) out[0] = acc;
}


// vote-like: vote_info[v] = {beg, cnt} -> per member a 16-B meta {pay16, ...} -> payload; then a
// 16-B + 8-B store per lane (the consensus write)
__global__ void k_gather_meta(const uint8_t* __restrict__ pay, const int4* __restrict__ vinfo, const uint4* __restrict__ meta,
                              int64_t nf, uint8_t* __restrict__ outq, uint8_t* __restrict__ outs, int store, uint32_t* out) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int g = lane / CH, c = lane - g * CH;
    const int64_t fi = wave * FPW + g;
    uint32_t acc = 0;
    if (g < FPW && fi < nf) {
        const int4 vi = vinfo[fi];
        const int32_t b = vi.x, n = vi.y;
        for (int k0 = 0; k0 < n; k0 += 4) {
            uint4 m[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) m[u] = (k0 + u < n) ? meta[b + k0 + u] : make_uint4(0, 0, 0, 0);
            uint4 q[4]; uint2 s[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                q[u] = make_uint4(0, 0, 0, 0); s[u] = make_uint2(0, 0);
                if (k0 + u < n) {
                    const uint8_t* r = pay + ((int64_t)m[u].x << 4);
                    q[u] = *reinterpret_cast<const uint4*>(r + 16 * c);
                    s[u] = *reinterpret_cast<const uint2*>(r + 160 + 8 * c);
                }
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) acc += q[u].x ^ q[u].y ^ q[u].z ^ q[u].w ^ s[u].x ^ s[u].y;
        }
        if (store) {
            *reinterpret_cast<uint4*>(outq + fi * 160 + 16 * c) = make_uint4(acc, acc, acc, acc);
            *reinterpret_cast<uint2*>(outs + fi * 80 + 8 * c) = make_uint2(acc, acc);
        }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

int main() {
    const int64_t nrec = 20000000;
    std::mt19937_64 rng(7);
    std::poisson_distribution<int> pois(3.4);
    std::vector<int32_t> beg, cnt;
    for (int64_t r = 0; r < nrec;) {
        int n = 1 + pois(rng);
        if (r + n > nrec) n = (int)(nrec - r);
        beg.push_back((int32_t)r); cnt.push_back(n); r += n;
    }
    const int64_t nf = beg.size();
    std::vector<int32_t> order(nf), shuf(nf);
    for (int64_t i = 0; i < nf; ++i) order[i] = shuf[i] = (int32_t)i;
    // shuffled within windows of 64k families (emission order is roughly positional)
    for (int64_t i = 0; i < nf; i += 65536) std::shuffle(shuf.begin() + i, shuf.begin() + std::min(nf, i + 65536), rng);
    const int64_t nblk = (nrec + 255) / 256;
    std::vector<int32_t> first(nblk + 1);
    { int64_t f = 0; for (int64_t b = 0; b <= nblk; ++b) { while (f < nf && beg[f] < b * 256) ++f; first[b] = (int32_t)f; } }
    uint8_t* pay; int32_t *d_beg, *d_cnt, *d_ord, *d_shuf, *d_first; uint32_t* d_out;
    CK(hipMalloc(&pay, nrec * SLOT)); CK(hipMemset(pay, 1, nrec * SLOT));
    CK(hipMalloc(&d_beg, nf * 4)); CK(hipMalloc(&d_cnt, nf * 4)); CK(hipMalloc(&d_ord, nf * 4)); CK(hipMalloc(&d_shuf, nf * 4));
    CK(hipMalloc(&d_first, (nblk + 1) * 4)); CK(hipMalloc(&d_out, 4));
    CK(hipMemcpy(d_beg, beg.data(), nf * 4, hipMemcpyHostToDevice)); CK(hipMemcpy(d_cnt, cnt.data(), nf * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_ord, order.data(), nf * 4, hipMemcpyHostToDevice)); CK(hipMemcpy(d_shuf, shuf.data(), nf * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_first, first.data(), (nblk + 1) * 4, hipMemcpyHostToDevice));
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    const double bytes = (double)nrec * 240.0;
    auto run = [&](const char* name, auto launch) {
        for (int w = 0; w < 2; ++w) launch();
        CK(hipEventRecord(a)); for (int i = 0; i < 5; ++i) launch(); CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b)); ms /= 5;
        printf("%-10s %8.3f ms  %7.1f GB/s (240 B/record)\n", name, ms, bytes / ms / 1e6);
    };
    const int64_t waves = (nf + FPW - 1) / FPW;
    run("stream", [&] { k_stream<<<4096, 256>>>((const uint4*)pay, nrec * SLOT / 16, d_out); });
    run("gather", [&] { k_gather<<<(waves + 3) / 4, 256>>>(pay, d_ord, d_beg, d_cnt, nf, d_out); });
    run("gather_p", [&] { k_gather<<<(waves + 3) / 4, 256>>>(pay, d_shuf, d_beg, d_cnt, nf, d_out); });
    std::vector<int4> vinfo(nf); std::vector<uint4> meta(nrec);
    for (int64_t f = 0; f < nf; ++f) vinfo[f] = make_int4(beg[f], cnt[f], 0, 0);
    for (int64_t r = 0; r < nrec; ++r) meta[r] = make_uint4((uint32_t)(r * SLOT / 16), 0, 150, 0);
    int4* d_vi; uint4* d_meta; uint8_t *oq, *os;
    CK(hipMalloc(&d_vi, nf * 16)); CK(hipMalloc(&d_meta, nrec * 16)); CK(hipMalloc(&oq, nf * 160)); CK(hipMalloc(&os, nf * 80));
    CK(hipMemcpy(d_vi, vinfo.data(), nf * 16, hipMemcpyHostToDevice)); CK(hipMemcpy(d_meta, meta.data(), nrec * 16, hipMemcpyHostToDevice));
    run("meta", [&] { k_gather_meta<<<(waves + 3) / 4, 256>>>(pay, d_vi, d_meta, nf, oq, os, 0, d_out); });
    run("meta+st", [&] { k_gather_meta<<<(waves + 3) / 4, 256>>>(pay, d_vi, d_meta, nf, oq, os, 1, d_out); });
    run("lds", [&] { k_lds<<<nblk, 256, 256 * SLOT>>>(pay, d_first, d_beg, d_cnt, nrec, nf, d_out); });
    CK(hipDeviceSynchronize());
    printf("families %lld\n", (long long)nf);
    return 0;
}
