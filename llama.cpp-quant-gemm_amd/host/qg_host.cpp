// qg_host.cpp — libqg_host.so: host-only twins of the reference's CPU entry points
// (include/qg/qg_host.h). Plain C++17 on the host, no HIP; built with -ffp-contract=off so every
// float operation is the single IEEE rounding the reference's scalar loops perform.
//
// Layout: a weight format is a traits struct (block bytes, field offsets, per-block formula); the
// GEMM walks output rows (optionally over a persistent worker pool — each output's summation stays
// serial in block order, so the thread count never changes a bit). Half <-> float goes through the F16C
// conversion instructions (round-to-nearest-even, as cuda_fp16's __float2half).
#include <immintrin.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/qg/blocks.h"
#include "../../include/qg/qg.h"
#include "../../include/qg/qg_host.h"

namespace {

__attribute__((target("f16c"))) inline float half_to_float(const uint8_t* p) {
    uint16_t h;
    memcpy(&h, p, 2);
    return _cvtsh_ss(h);
}
__attribute__((target("f16c"))) inline uint16_t float_to_half(float f) {
    return _cvtss_sh(f, _MM_FROUND_TO_NEAREST_INT);
}

constexpr int QK = 32;

// Q8_1 activation block: ds = (d, s) halves at 0 / 2, qs at 4 (include/quant_types.h:116-121).
struct ActBlock {
    float d, s;
    const int8_t* qs;
    explicit ActBlock(const uint8_t* p)
        : d(half_to_float(p)), s(half_to_float(p + 2)), qs(reinterpret_cast<const int8_t*>(p + 4)) {}
};

// Weight formats. `value(p, e)` is element e's stored integer (no offset removed), `term` the
// per-block fp32 formula in the reference's operation order (see qg_common.hpp's header).
struct FmtQ4_0 {
    static constexpr int bytes = 18;
    static int value(const uint8_t* p, int e) { return e < 16 ? (p[2 + e] & 0x0F) : (p[2 + e - 16] >> 4); }
    static float term(const uint8_t* p, int32_t sumi, const ActBlock& a) {
        const float dw = half_to_float(p);
        return dw * (a.d * (float)sumi - 8.0f * a.s);  // include/gemm_reference.h:216
    }
};
struct FmtQ4_1 {
    static constexpr int bytes = 20;
    static int value(const uint8_t* p, int e) { return e < 16 ? (p[4 + e] & 0x0F) : (p[4 + e - 16] >> 4); }
    static float term(const uint8_t* p, int32_t sumi, const ActBlock& a) {
        const float dw = half_to_float(p), mw = half_to_float(p + 2);
        return dw * a.d * (float)sumi + mw * a.s;  // d * d8 * sumi + m * s8 (no /4)
    }
};
template <int QH, int QS> inline int q5_value(const uint8_t* p, int e) {
    uint32_t qh;
    memcpy(&qh, p + QH, 4);
    const int nib = e < 16 ? (p[QS + e] & 0x0F) : (p[QS + e - 16] >> 4);
    return nib | (int)(((qh >> e) & 1u) << 4);
}
struct FmtQ5_0 {
    static constexpr int bytes = 22;
    static int value(const uint8_t* p, int e) { return q5_value<2, 6>(p, e); }
    static float term(const uint8_t* p, int32_t sumi, const ActBlock& a) {
        const float dw = half_to_float(p);
        return dw * (a.d * (float)sumi - 16.0f * a.s);
    }
};
struct FmtQ5_1 {
    static constexpr int bytes = 24;
    static int value(const uint8_t* p, int e) { return q5_value<4, 8>(p, e); }
    static float term(const uint8_t* p, int32_t sumi, const ActBlock& a) {
        const float dw = half_to_float(p), mw = half_to_float(p + 2);
        return dw * a.d * (float)sumi + mw * a.s;
    }
};
struct FmtQ8_0 {
    static constexpr int bytes = 34;
    static int value(const uint8_t* p, int e) { return (int)(int8_t)p[2 + e]; }
    static float term(const uint8_t* p, int32_t sumi, const ActBlock& a) {
        const float dw = half_to_float(p);
        return (float)sumi * a.d * dw;  // include/gemm_reference.h:260
    }
};

template <class F> inline int32_t block_sumi(const uint8_t* w, const ActBlock& a) {
    // element pairs (k, k + 16) in the reference's loop order (integer sums are order-free anyway);
    // constant indices, so the per-format branches fold away
    int32_t sumi = 0;
    for (int k = 0; k < QK / 2; ++k)
        sumi += (int32_t)a.qs[k] * F::value(w, k) + (int32_t)a.qs[k + QK / 2] * F::value(w, k + QK / 2);
    return sumi;
}

template <class F> void gemm_rows(const uint8_t* A, const uint8_t* B, float* C, int M, int N, int K, int j0, int j1) {
    const int nb = K / QK;
    const size_t arow = (size_t)nb * 36, wrow = (size_t)nb * F::bytes;
    for (int i = 0; i < M; ++i)
        for (int j = j0; j < j1; ++j) {
            float sum = 0.0f;
            for (int b = 0; b < nb; ++b) {
                const ActBlock a(A + i * arow + (size_t)b * 36);
                const uint8_t* w = B + j * wrow + (size_t)b * F::bytes;
                sum += F::term(w, block_sumi<F>(w, a), a);
            }
            C[(size_t)i * N + j] = sum;
        }
}

// Process-wide persistent worker pool: threads are started once (grown on demand) and parked on
// a condition variable between jobs, so a multi-threaded call costs one wake-up per worker instead
// of a thread start and join (which dominated a 1-9 ms GEMV at 256 threads). One job at a time
// (callers are serialised by run_mu); the calling thread takes part 0.
class Pool {
  public:
    static Pool& get() {
        static Pool p;
        return p;
    }
    void run(int parts, const std::function<void(int)>& fn) {
        std::lock_guard<std::mutex> serial(run_mu_);
        grow(parts - 1);
        {
            std::lock_guard<std::mutex> lk(mu_);
            job_ = &fn;
            parts_ = parts;
            pending_ = parts - 1;
            ++gen_;
        }
        cv_.notify_all();
        fn(0);
        std::unique_lock<std::mutex> lk(mu_);
        done_.wait(lk, [&] { return pending_ == 0; });
        job_ = nullptr;
    }
    ~Pool() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : workers_) t.join();
    }

  private:
    void grow(int n) {
        while ((int)workers_.size() < n) {
            const int id = (int)workers_.size() + 1;  // part index this worker takes
            workers_.emplace_back([this, id] { loop(id); });
        }
    }
    void loop(int id) {
        unsigned long long seen = 0;
        for (;;) {
            const std::function<void(int)>* job;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
                if (stop_) return;
                seen = gen_;
                if (id >= parts_) continue;  // not needed for this job
                job = job_;
            }
            (*job)(id);
            std::lock_guard<std::mutex> lk(mu_);
            if (--pending_ == 0) done_.notify_one();
        }
    }
    std::mutex run_mu_, mu_;
    std::condition_variable cv_, done_;
    std::vector<std::thread> workers_;
    const std::function<void(int)>* job_ = nullptr;
    int parts_ = 0, pending_ = 0;
    unsigned long long gen_ = 0;
    bool stop_ = false;
};

template <class F> void gemm_threads(const void* A, const void* B, float* C, int M, int N, int K, int threads) {
    auto run = [&](int j0, int j1) {
        gemm_rows<F>((const uint8_t*)A, (const uint8_t*)B, C, M, N, K, j0, j1);
    };
    threads = std::max(1, std::min(threads, N));
    if (threads == 1) return run(0, N);
    const int per = (N + threads - 1) / threads;
    const std::function<void(int)> part = [&](int t) {
        const int j0 = t * per, j1 = std::min(N, j0 + per);
        if (j0 < j1) run(j0, j1);
    };
    Pool::get().run(threads, part);
}

int check_gemm(const void* A, const void* B, const float* C, int M, int N, int K) {
    if (M < 0 || N < 0) return QG_ERR_INVALID_ARG;
    if (K <= 0 || K % QK != 0) return QG_ERR_BAD_K;
    if ((M > 0 && N > 0) && (!A || !B || !C)) return QG_ERR_INVALID_ARG;
    return QG_OK;
}

}  // namespace

extern "C" {

int qg_gemm_w4a8_cpu_mt(const void* A, const void* B, float* C, int M, int N, int K, int wtype, int threads) {
    const int rc = check_gemm(A, B, C, M, N, K);
    if (rc != QG_OK) return rc;
    if (M == 0 || N == 0) return QG_OK;
    switch (wtype) {
        case QG_TYPE_Q4_0: gemm_threads<FmtQ4_0>(A, B, C, M, N, K, threads); return QG_OK;
        case QG_TYPE_Q4_1: gemm_threads<FmtQ4_1>(A, B, C, M, N, K, threads); return QG_OK;
        case QG_TYPE_Q5_0: gemm_threads<FmtQ5_0>(A, B, C, M, N, K, threads); return QG_OK;
        case QG_TYPE_Q5_1: gemm_threads<FmtQ5_1>(A, B, C, M, N, K, threads); return QG_OK;
        case QG_TYPE_Q8_0: gemm_threads<FmtQ8_0>(A, B, C, M, N, K, threads); return QG_OK;
    }
    return QG_ERR_UNSUPPORTED;
}

int qg_gemm_w4a8_q4_0_cpu(const void* A, const void* B, float* C, int M, int N, int K) {
    return qg_gemm_w4a8_cpu_mt(A, B, C, M, N, K, QG_TYPE_Q4_0, 1);
}

int qg_gemm_w8a8_cpu(const void* A, const void* B, float* C, int M, int N, int K) {
    return qg_gemm_w4a8_cpu_mt(A, B, C, M, N, K, QG_TYPE_Q8_0, 1);
}

void qg_vec_dot_q4_0_q8_1_cpu(int n, float* s, const void* vx, const void* vy) {
    const uint8_t* x = (const uint8_t*)vx;
    const uint8_t* y = (const uint8_t*)vy;
    float sum = 0.0f;
    for (int b = 0; b < n / QK; ++b) {
        const ActBlock a(y + (size_t)b * 36);
        const uint8_t* w = x + (size_t)b * FmtQ4_0::bytes;
        sum += FmtQ4_0::term(w, block_sumi<FmtQ4_0>(w, a), a);
    }
    *s = sum;
}

void qg_vec_dot_q8_0_q8_1_cpu(int n, float* s, const void* vx, const void* vy) {
    const uint8_t* x = (const uint8_t*)vx;
    const uint8_t* y = (const uint8_t*)vy;
    float sum = 0.0f;
    for (int b = 0; b < n / QK; ++b) {
        const ActBlock a(y + (size_t)b * 36);
        const uint8_t* w = x + (size_t)b * FmtQ8_0::bytes;
        const float dw = half_to_float(w);
        sum += (float)block_sumi<FmtQ8_0>(w, a) * dw * a.d;  // sumi * d_w * d_a (gemm_reference.h:333)
    }
    *s = sum;
}

int qg_gemm_fp32_cpu(const float* A, const float* B, float* C, int M, int N, int K) {
    if (M < 0 || N < 0 || K < 0) return QG_ERR_INVALID_ARG;
    if (M == 0 || N == 0) return QG_OK;
    if (!A || !B || !C) return QG_ERR_INVALID_ARG;
    for (int i = 0; i < M; ++i)
        for (int j = 0; j < N; ++j) {
            float sum = 0.0f;
            for (int k = 0; k < K; ++k) sum += A[(size_t)i * K + k] * B[(size_t)j * K + k];
            C[(size_t)i * N + j] = sum;
        }
    return QG_OK;
}

int qg_quantize_row_q8_1_cpu(const float* x, void* yv, int64_t k) {
    if (k < 0 || k % QK != 0) return QG_ERR_BAD_K;
    if (k && (!x || !yv)) return QG_ERR_INVALID_ARG;
    uint8_t* y = (uint8_t*)yv;
    for (int64_t b = 0; b < k / QK; ++b) {
        const float* v = x + b * QK;
        uint8_t* o = y + b * 36;
        float amax = 0.0f, sum = 0.0f;
        for (int j = 0; j < QK; ++j) {
            amax = std::max(amax, std::fabs(v[j]));
            sum += v[j];
        }
        const float d = amax / 127.0f;
        const uint16_t hd = float_to_half(d), hs = float_to_half(sum);
        memcpy(o, &hd, 2);
        memcpy(o + 2, &hs, 2);
        const float id = d > 0 ? 1.0f / d : 0.0f;
        for (int j = 0; j < QK; ++j) {
            const int q = (int)std::round(v[j] * id);  // roundf: half away from zero
            o[4 + j] = (uint8_t)(int8_t)std::max(-128, std::min(127, q));
        }
    }
    return QG_OK;
}

int qg_quantize_row_q4_0_cpu(const float* x, void* yv, int64_t k) {
    if (k < 0 || k % QK != 0) return QG_ERR_BAD_K;
    if (k && (!x || !yv)) return QG_ERR_INVALID_ARG;
    uint8_t* y = (uint8_t*)yv;
    for (int64_t b = 0; b < k / QK; ++b) {
        const float* v = x + b * QK;
        uint8_t* o = y + b * 18;
        float amax = 0.0f;
        for (int j = 0; j < QK; ++j) amax = std::max(amax, std::fabs(v[j]));
        const float d = amax / 7.0f;
        const uint16_t hd = float_to_half(d);
        memcpy(o, &hd, 2);
        const float id = d > 0 ? 1.0f / d : 0.0f;
        auto q4 = [&](float f) { return std::max(0, std::min(15, (int)std::round(f * id) + 8)); };
        for (int j = 0; j < QK / 2; ++j) o[2 + j] = (uint8_t)(q4(v[j]) | (q4(v[j + QK / 2]) << 4));
    }
    return QG_OK;
}

int qg_fill_step4_cpu(unsigned seed, int M, int N, int K, int row0, int row1, float* a, float* b) {
    if (M < 0 || N < 0 || K < 0 || row0 < 0 || row1 < row0 || row1 > N) return QG_ERR_INVALID_ARG;
    auto draw = []() { return 2.0f * (float)rand() / RAND_MAX - 1.0f; };
    srand(seed);
    const int64_t na = (int64_t)M * K;
    for (int64_t i = 0; i < na; ++i) {
        const float v = draw();
        if (a) a[i] = v;
    }
    const int64_t skip = (int64_t)row0 * K, take = (int64_t)(row1 - row0) * K;
    for (int64_t i = 0; i < skip; ++i) (void)rand();
    for (int64_t i = 0; i < take; ++i) {
        const float v = draw();
        if (b) b[i] = v;
    }
    return QG_OK;
}

}  // extern "C"
