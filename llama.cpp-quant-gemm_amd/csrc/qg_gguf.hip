// qg_gguf.hip — GGUF reader (host code): the weight-file side of the ggml-facing adapter
// (SURVEY.md §8f-4). Q4_0 / Q4_1 / Q5_0 / Q5_1 / Q8_0 tensors in GGUF files use the same block
// bytes as the kernels (qg/blocks.h), so a tensor's data is uploaded as-is and viewed as a
// qg_tensor_view for qg_gemm_w4a8_from_view.
//
// Format (GGUF v2/v3, little-endian): "GGUF", u32 version, u64 tensor count, u64 metadata count;
// metadata key/value pairs (string = u64 length + bytes; typed values, arrays of values); tensor
// infos (name, u32 n_dims, u64 ne[n_dims], u32 ggml type, u64 offset relative to the data section);
// the data section starts at the next multiple of general.alignment (default 32).
// The file is mapped read-only; nothing is executed from it, every length and offset is checked
// against the file size before use.
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <string>
#include <vector>

#include "../../include/qg/qg.h"

struct qg_gguf {
    int fd = -1;
    const uint8_t* map = nullptr;
    size_t size = 0;
    uint32_t version = 0;
    uint64_t alignment = 32;
    uint64_t data_start = 0;
    struct kv_t {
        std::string key;
        uint32_t type;
        uint64_t off;     // file offset of the value
        uint64_t count;   // arrays: element count
        uint32_t elem;    // arrays: element type
    };
    struct tensor_t {
        std::string name;
        uint32_t n_dims;
        int64_t ne[4];
        uint32_t type;
        uint64_t offset;  // relative to data_start
        uint64_t nbytes;
    };
    std::vector<kv_t> kvs;
    std::vector<tensor_t> tensors;
};

namespace {
enum : uint32_t { T_U8 = 0, T_I8, T_U16, T_I16, T_U32, T_I32, T_F32, T_BOOL, T_STR, T_ARR, T_U64, T_I64, T_F64 };

struct reader {
    const uint8_t* p;
    size_t size, pos = 0;
    bool ok = true;
    bool need(uint64_t n) {
        if (!ok || n > size - pos) ok = false;
        return ok;
    }
    template <class T> T get() {
        T v{};
        if (need(sizeof(T))) { memcpy(&v, p + pos, sizeof(T)); pos += sizeof(T); }
        return v;
    }
    std::string str() {
        const uint64_t n = get<uint64_t>();
        if (!need(n)) return {};
        std::string s((const char*)p + pos, (size_t)n);
        pos += n;
        return s;
    }
    void skip(uint64_t n) { if (need(n)) pos += n; }
};

uint64_t scalar_size(uint32_t t) {
    switch (t) {
        case T_U8: case T_I8: case T_BOOL: return 1;
        case T_U16: case T_I16: return 2;
        case T_U32: case T_I32: case T_F32: return 4;
        case T_U64: case T_I64: case T_F64: return 8;
    }
    return 0;
}

// skip one value of type t (strings and nested arrays included)
void skip_value(reader& r, uint32_t t, int depth = 0) {
    if (t == T_STR) { r.str(); return; }
    if (t == T_ARR) {
        if (depth > 4) { r.ok = false; return; }
        const uint32_t et = r.get<uint32_t>();
        const uint64_t n = r.get<uint64_t>();
        if (et == T_STR || et == T_ARR) {
            for (uint64_t i = 0; i < n && r.ok; ++i) skip_value(r, et, depth + 1);
        } else {
            const uint64_t s = scalar_size(et);
            if (s == 0 || (n != 0 && s > UINT64_MAX / n)) { r.ok = false; return; }
            r.skip(n * s);
        }
        return;
    }
    const uint64_t s = scalar_size(t);
    if (s == 0) { r.ok = false; return; }
    r.skip(s);
}

// bytes of a tensor of ggml type t with ne elements per row-major dims (0 if unsupported)
uint64_t tensor_bytes(uint32_t t, const int64_t ne[4], uint32_t n_dims) {
    uint64_t n = 1;
    for (uint32_t d = 0; d < n_dims; ++d) {
        if (ne[d] < 0 || (ne[d] != 0 && n > UINT64_MAX / (uint64_t)ne[d])) return 0;
        n *= (uint64_t)ne[d];
    }
    switch (t) {
        case QG_TYPE_F32: return n * 4;
        case QG_TYPE_F16: return n * 2;
    }
    const int bb = qg_block_bytes((int)t);
    if (bb == 0 || ne[0] % 32 != 0) return 0;
    return n / 32 * (uint64_t)bb;
}

int parse(qg_gguf* g) {
    reader r{g->map, g->size};
    if (r.get<uint32_t>() != 0x46554747u) return QG_ERR_INVALID_ARG;  // "GGUF"
    g->version = r.get<uint32_t>();
    if (g->version < 2 || g->version > 3) return QG_ERR_UNSUPPORTED;
    const uint64_t n_tensors = r.get<uint64_t>();
    const uint64_t n_kv = r.get<uint64_t>();
    if (!r.ok || n_tensors > (1u << 24) || n_kv > (1u << 24)) return QG_ERR_INVALID_ARG;
    for (uint64_t i = 0; i < n_kv && r.ok; ++i) {
        qg_gguf::kv_t kv;
        kv.key = r.str();
        kv.type = r.get<uint32_t>();
        kv.count = 0;
        kv.elem = 0;
        if (kv.type == T_ARR) {
            const size_t save = r.pos;
            kv.elem = r.get<uint32_t>();
            kv.count = r.get<uint64_t>();
            r.pos = save;
        }
        kv.off = r.pos;
        skip_value(r, kv.type);
        if (!r.ok) break;
        if (kv.key == "general.alignment" && (kv.type == T_U32 || kv.type == T_I32)) {
            uint32_t a;
            memcpy(&a, g->map + kv.off, 4);
            if (a == 0 || (a & (a - 1)) != 0) return QG_ERR_INVALID_ARG;
            g->alignment = a;
        }
        g->kvs.push_back(std::move(kv));
    }
    for (uint64_t i = 0; i < n_tensors && r.ok; ++i) {
        qg_gguf::tensor_t t;
        t.name = r.str();
        t.n_dims = r.get<uint32_t>();
        if (t.n_dims < 1 || t.n_dims > 4) return QG_ERR_UNSUPPORTED;
        for (int d = 0; d < 4; ++d) t.ne[d] = 1;
        for (uint32_t d = 0; d < t.n_dims; ++d) t.ne[d] = (int64_t)r.get<uint64_t>();
        t.type = r.get<uint32_t>();
        t.offset = r.get<uint64_t>();
        t.nbytes = tensor_bytes(t.type, t.ne, t.n_dims);
        g->tensors.push_back(std::move(t));
    }
    if (!r.ok) return QG_ERR_INVALID_ARG;
    g->data_start = (r.pos + g->alignment - 1) / g->alignment * g->alignment;
    for (auto& t : g->tensors) {
        if (t.offset % g->alignment != 0) return QG_ERR_INVALID_ARG;
        if (t.nbytes != 0 && (g->data_start > g->size || t.offset > g->size - g->data_start ||
                              t.nbytes > g->size - g->data_start - t.offset))
            return QG_ERR_INVALID_ARG;  // data past the end of the file
    }
    return QG_OK;
}
}  // namespace

extern "C" {

int qg_gguf_open(const char* path, qg_gguf** out) {
    if (!path || !out) return QG_ERR_INVALID_ARG;
    *out = nullptr;
    const int fd = open(path, O_RDONLY | O_CLOEXEC);
    if (fd < 0) return QG_ERR_INVALID_ARG;
    struct stat st;
    if (fstat(fd, &st) != 0 || st.st_size < 24) { close(fd); return QG_ERR_INVALID_ARG; }
    void* m = mmap(nullptr, (size_t)st.st_size, PROT_READ, MAP_PRIVATE, fd, 0);
    if (m == MAP_FAILED) { close(fd); return QG_ERR_INVALID_ARG; }
    qg_gguf* g = new qg_gguf;
    g->fd = fd;
    g->map = (const uint8_t*)m;
    g->size = (size_t)st.st_size;
    const int rc = parse(g);
    if (rc != QG_OK) { qg_gguf_close(g); return rc; }
    *out = g;
    return QG_OK;
}

void qg_gguf_close(qg_gguf* g) {
    if (!g) return;
    if (g->map) munmap((void*)g->map, g->size);
    if (g->fd >= 0) close(g->fd);
    delete g;
}

int qg_gguf_version(const qg_gguf* g) { return g ? (int)g->version : -1; }
int64_t qg_gguf_alignment(const qg_gguf* g) { return g ? (int64_t)g->alignment : -1; }
int64_t qg_gguf_tensor_count(const qg_gguf* g) { return g ? (int64_t)g->tensors.size() : -1; }
int64_t qg_gguf_kv_count(const qg_gguf* g) { return g ? (int64_t)g->kvs.size() : -1; }

int64_t qg_gguf_find_tensor(const qg_gguf* g, const char* name) {
    if (!g || !name) return -1;
    for (size_t i = 0; i < g->tensors.size(); ++i)
        if (g->tensors[i].name == name) return (int64_t)i;
    return -1;
}

int qg_gguf_tensor_info(const qg_gguf* g, int64_t i, const char** name, int* type, int* n_dims, int64_t ne[4],
                        uint64_t* nbytes) {
    if (!g || i < 0 || i >= (int64_t)g->tensors.size()) return QG_ERR_INVALID_ARG;
    const auto& t = g->tensors[(size_t)i];
    if (name) *name = t.name.c_str();
    if (type) *type = (int)t.type;
    if (n_dims) *n_dims = (int)t.n_dims;
    if (ne) for (int d = 0; d < 4; ++d) ne[d] = t.ne[d];
    if (nbytes) *nbytes = t.nbytes;
    return QG_OK;
}

const void* qg_gguf_tensor_data(const qg_gguf* g, int64_t i) {
    if (!g || i < 0 || i >= (int64_t)g->tensors.size() || g->tensors[(size_t)i].nbytes == 0) return nullptr;
    return g->map + g->data_start + g->tensors[(size_t)i].offset;
}

int qg_gguf_upload_tensor(const qg_gguf* g, int64_t i, void* dst, size_t dst_bytes, qg_stream_t stream) {
    const void* src = qg_gguf_tensor_data(g, i);
    if (!src || !dst) return QG_ERR_INVALID_ARG;
    const uint64_t n = g->tensors[(size_t)i].nbytes;
    if (dst_bytes < n) return QG_ERR_INVALID_ARG;
    // pageable source: the copy is staged by the runtime; synchronous with respect to the host
    hipError_t e = hipMemcpyAsync(dst, src, (size_t)n, hipMemcpyHostToDevice, (hipStream_t)stream);
    if (e == hipSuccess) e = hipStreamSynchronize((hipStream_t)stream);
    return e == hipSuccess ? QG_OK : QG_ERR_HIP;
}

int qg_gguf_tensor_view(const qg_gguf* g, int64_t i, void* device_data, qg_tensor_view* out) {
    if (!g || !out || i < 0 || i >= (int64_t)g->tensors.size()) return QG_ERR_INVALID_ARG;
    const auto& t = g->tensors[(size_t)i];
    if (t.nbytes == 0) return QG_ERR_UNSUPPORTED;
    out->data = device_data;
    out->type = (int)t.type;
    for (int d = 0; d < 4; ++d) out->ne[d] = t.ne[d];
    // ggml byte strides: nb[0] = element / block size, nb[1] = row bytes, then dense
    const int bb = qg_block_bytes((int)t.type);
    const size_t row = t.type == QG_TYPE_F32 ? (size_t)t.ne[0] * 4
                       : t.type == QG_TYPE_F16 ? (size_t)t.ne[0] * 2
                                               : (size_t)(t.ne[0] / 32) * (size_t)bb;
    out->nb[0] = t.type == QG_TYPE_F32 ? 4 : t.type == QG_TYPE_F16 ? 2 : (size_t)bb;
    out->nb[1] = row;
    out->nb[2] = row * (size_t)t.ne[1];
    out->nb[3] = out->nb[2] * (size_t)t.ne[2];
    return QG_OK;
}

int qg_gguf_kv_info(const qg_gguf* g, int64_t i, const char** key, int* type, uint64_t* array_count,
                    int* array_type) {
    if (!g || i < 0 || i >= (int64_t)g->kvs.size()) return QG_ERR_INVALID_ARG;
    const auto& kv = g->kvs[(size_t)i];
    if (key) *key = kv.key.c_str();
    if (type) *type = (int)kv.type;
    if (array_count) *array_count = kv.count;
    if (array_type) *array_type = (int)kv.elem;
    return QG_OK;
}

int64_t qg_gguf_find_kv(const qg_gguf* g, const char* key) {
    if (!g || !key) return -1;
    for (size_t i = 0; i < g->kvs.size(); ++i)
        if (g->kvs[i].key == key) return (int64_t)i;
    return -1;
}

// Scalar values as int64 / double; strings as (pointer into the mapping, length).
int qg_gguf_kv_int(const qg_gguf* g, int64_t i, int64_t* v) {
    if (!g || !v || i < 0 || i >= (int64_t)g->kvs.size()) return QG_ERR_INVALID_ARG;
    const auto& kv = g->kvs[(size_t)i];
    const uint8_t* p = g->map + kv.off;
    switch (kv.type) {
        case T_U8: *v = *p; return QG_OK;
        case T_I8: *v = (int8_t)*p; return QG_OK;
        case T_BOOL: *v = *p != 0; return QG_OK;
        case T_U16: { uint16_t x; memcpy(&x, p, 2); *v = x; return QG_OK; }
        case T_I16: { int16_t x; memcpy(&x, p, 2); *v = x; return QG_OK; }
        case T_U32: { uint32_t x; memcpy(&x, p, 4); *v = x; return QG_OK; }
        case T_I32: { int32_t x; memcpy(&x, p, 4); *v = x; return QG_OK; }
        case T_U64: { uint64_t x; memcpy(&x, p, 8); *v = (int64_t)x; return QG_OK; }
        case T_I64: { int64_t x; memcpy(&x, p, 8); *v = x; return QG_OK; }
    }
    return QG_ERR_UNSUPPORTED;
}

int qg_gguf_kv_float(const qg_gguf* g, int64_t i, double* v) {
    if (!g || !v || i < 0 || i >= (int64_t)g->kvs.size()) return QG_ERR_INVALID_ARG;
    const auto& kv = g->kvs[(size_t)i];
    if (kv.type == T_F32) { float x; memcpy(&x, g->map + kv.off, 4); *v = x; return QG_OK; }
    if (kv.type == T_F64) { memcpy(v, g->map + kv.off, 8); return QG_OK; }
    int64_t x;
    const int rc = qg_gguf_kv_int(g, i, &x);
    if (rc == QG_OK) *v = (double)x;
    return rc;
}

int qg_gguf_kv_string(const qg_gguf* g, int64_t i, const char** s, uint64_t* len) {
    if (!g || !s || !len || i < 0 || i >= (int64_t)g->kvs.size()) return QG_ERR_INVALID_ARG;
    const auto& kv = g->kvs[(size_t)i];
    if (kv.type != T_STR) return QG_ERR_UNSUPPORTED;
    memcpy(len, g->map + kv.off, 8);
    *s = (const char*)g->map + kv.off + 8;
    return QG_OK;
}

}  // extern "C"
