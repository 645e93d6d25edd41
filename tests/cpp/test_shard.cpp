// test_shard.cpp — C++ caller of the row-sharded multi-GPU entry (include/qg/qg_shard.h) the way a
// llama.cpp-style host would use it: the caller creates one RCCL communicator per device
// (ncclCommInitAll, one thread per device), each rank keeps its contiguous weight rows resident
// and calls qg_sharded_gemm_w4a8 on its own stream; every rank ends with the full C[M][N].
// Checked against the single-GPU qg_gemm_w4a8 on the whole B (bit-identical on the GEMV path,
// M <= 4; reassociation-level agreement is the MFMA path's bar, checked loosely here and exactly in
// tests/test_gpu_shard.py). Usage: test_shard [ndev] (default: every visible GPU; the GPU box has 1).
// Exit status 0 = parity held. Built and run by tests/test_cpp_driver.py.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <thread>
#include <vector>

#include "qg/qg.h"
#include "qg/qg_shard.h"

#define HCK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(2); } } while (0)
#define QCK(x) do { int r_ = (x); if (r_ != QG_OK) { fprintf(stderr, "qg status %d (%s) @%d nccl %d\n", r_, qg_status_string(r_), __LINE__, qg_shard_last_nccl_error()); exit(3); } } while (0)

// host data: deterministic Q8_1 / Q4_0 blocks from the device quantizers of device 0
struct Problem {
    int M, N, K;
    std::vector<uint8_t> aq, bq;  // [M][K/32][36], [N][K/32][18]
    std::vector<float> ref;       // single-GPU qg_gemm_w4a8 on the whole B
};

static Problem make_problem(int M, int N, int K, unsigned seed) {
    Problem p{M, N, K, {}, {}, {}};
    std::vector<float> a((size_t)M * K), b((size_t)N * K);
    srand(seed);
    for (auto& v : a) v = 2.0f * (float)rand() / (float)RAND_MAX - 1.0f;
    for (auto& v : b) v = 2.0f * (float)rand() / (float)RAND_MAX - 1.0f;
    const size_t nb = K / 32;
    p.aq.resize((size_t)M * nb * 36);
    p.bq.resize((size_t)N * nb * 18);
    p.ref.resize((size_t)M * N);
    HCK(hipSetDevice(0));
    float *da, *db, *dc;
    void *dA, *dB;
    HCK(hipMalloc(&da, a.size() * 4));
    HCK(hipMalloc(&db, b.size() * 4));
    HCK(hipMalloc(&dA, p.aq.size()));
    HCK(hipMalloc(&dB, p.bq.size()));
    HCK(hipMalloc(&dc, p.ref.size() * 4));
    HCK(hipMemcpy(da, a.data(), a.size() * 4, hipMemcpyHostToDevice));
    HCK(hipMemcpy(db, b.data(), b.size() * 4, hipMemcpyHostToDevice));
    QCK(qg_quantize_q8_1(da, dA, (int64_t)a.size(), nullptr));
    QCK(qg_quantize_q4_0(db, dB, (int64_t)b.size(), nullptr));
    QCK(qg_gemm_w4a8(dA, dB, dc, M, N, K, QG_TYPE_Q4_0, nullptr));
    HCK(hipDeviceSynchronize());
    HCK(hipMemcpy(p.aq.data(), dA, p.aq.size(), hipMemcpyDeviceToHost));
    HCK(hipMemcpy(p.bq.data(), dB, p.bq.size(), hipMemcpyDeviceToHost));
    HCK(hipMemcpy(p.ref.data(), dc, p.ref.size() * 4, hipMemcpyDeviceToHost));
    HCK(hipFree(da)); HCK(hipFree(db)); HCK(hipFree(dA)); HCK(hipFree(dB)); HCK(hipFree(dc));
    return p;
}

// one rank: its shard resident on its device, the sharded call, the full C back to the host
static void rank_main(const Problem& p, int dev, ncclComm_t comm, std::vector<float>* out) {
    HCK(hipSetDevice(dev));
    int world = 0, rank = 0;
    QCK(qg_shard_comm_count((qg_nccl_comm_t)comm, &world));
    QCK(qg_shard_comm_rank((qg_nccl_comm_t)comm, &rank));
    int row0 = 0, rows = 0;
    QCK(qg_shard_rows(p.N, world, rank, &row0, &rows));
    const size_t rb = (size_t)(p.K / 32) * 18;
    void *dA, *dB = nullptr, *ws = nullptr;
    float* dC;
    HCK(hipMalloc(&dA, p.aq.size()));
    HCK(hipMemcpy(dA, p.aq.data(), p.aq.size(), hipMemcpyHostToDevice));
    if (rows > 0) {
        HCK(hipMalloc(&dB, rows * rb));
        HCK(hipMemcpy(dB, p.bq.data() + (size_t)row0 * rb, rows * rb, hipMemcpyHostToDevice));
    }
    HCK(hipMalloc(&dC, (size_t)p.M * p.N * 4));
    const size_t wsb = qg_sharded_gemm_workspace_size(p.M, p.N, world);
    if (wsb) HCK(hipMalloc(&ws, wsb));
    hipStream_t st;
    HCK(hipStreamCreate(&st));
    for (int rep = 0; rep < 3; ++rep)  // repeated calls reuse the buffers
        QCK(qg_sharded_gemm_w4a8(dA, dB, dC, p.M, p.N, p.K, QG_TYPE_Q4_0, ws, wsb, (qg_nccl_comm_t)comm,
                                 reinterpret_cast<qg_stream_t>(st)));
    HCK(hipStreamSynchronize(st));
    out->resize((size_t)p.M * p.N);
    HCK(hipMemcpy(out->data(), dC, out->size() * 4, hipMemcpyDeviceToHost));
    HCK(hipStreamDestroy(st));
    HCK(hipFree(dA)); if (dB) HCK(hipFree(dB)); HCK(hipFree(dC)); if (ws) HCK(hipFree(ws));
}

int main(int argc, char** argv) {
    int ndev = 0;
    HCK(hipGetDeviceCount(&ndev));
    if (argc > 1) ndev = atoi(argv[1]);
    if (ndev < 1) return 2;
    std::vector<int> devs(ndev);
    for (int i = 0; i < ndev; ++i) devs[i] = i;
    std::vector<ncclComm_t> comms(ndev);
    if (ncclCommInitAll(comms.data(), ndev, devs.data()) != ncclSuccess) {
        fprintf(stderr, "ncclCommInitAll failed\n");
        return 2;
    }
    int fails = 0;
    const int shapes[][3] = {{1, 4096, 4096}, {1, 32000, 4096}, {3, 4097, 1024}, {2, 37, 256}, {12, 1000, 2048}};
    for (auto& s : shapes) {
        const Problem p = make_problem(s[0], s[1], s[2], 42);
        std::vector<std::vector<float>> outs(ndev);
        std::vector<std::thread> th;
        for (int r = 0; r < ndev; ++r) th.emplace_back(rank_main, std::cref(p), devs[r], comms[r], &outs[r]);
        for (auto& t : th) t.join();
        double maxrel = 0.0;
        size_t nbits = 0;
        for (int r = 0; r < ndev; ++r)
            for (size_t i = 0; i < p.ref.size(); ++i) {
                if (memcmp(&outs[r][i], &p.ref[i], 4) != 0) ++nbits;
                maxrel = fmax(maxrel, fabs((double)outs[r][i] - p.ref[i]) / (fabs((double)p.ref[i]) + 1e-3));
            }
        const bool gemv = s[0] <= 4;
        const bool ok = gemv ? nbits == 0 : maxrel < 1e-4;
        printf("world %d M=%d N=%d K=%d: %zu outputs differ in bits, max rel %.3g -> %s\n", ndev, s[0], s[1], s[2], nbits,
               maxrel, ok ? "ok" : "FAIL");
        fails += !ok;
    }
    for (auto c : comms) ncclCommDestroy(c);
    return fails ? 1 : 0;
}
