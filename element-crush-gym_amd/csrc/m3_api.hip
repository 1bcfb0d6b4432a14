// m3_api.hip -- the C ABI of include/m3.h (kernels and launchers: m3_kernels.hpp).
#include "m3_kernels.hpp"

#include <string>

namespace {
thread_local std::string g_err;
}  // namespace

int set_err(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#ifdef M3_SPLIT_TU  // the launchers are instantiated in m3_inst.hip, one TU per configuration
namespace m3k {
M3_INSTANTIATE(extern template, CF_0)
M3_INSTANTIATE(extern template, CF_1)
#ifndef M3_HEADLINE_ONLY  // A/B builds of the two specialised shapes only (Makefile `variant-fast`)
M3_INSTANTIATE(extern template, CF_2)
M3_INSTANTIATE(extern template, CF_3)
M3_INSTANTIATE(extern template, CF_4)
M3_INSTANTIATE(extern template, CF_5)
#ifndef M3_NO_WIDE_FRAME  // (Makefile `variant-frame16`: no 32 x 32 frame)
M3_INSTANTIATE(extern template, CF_6)
M3_INSTANTIATE(extern template, CF_7)
M3_INSTANTIATE(extern template, CF_8)
M3_INSTANTIATE(extern template, CF_9)
#endif
#endif
}  // namespace m3k
#endif
using namespace m3k;

namespace {
// rows < columns: the last action ids decode to a swap with the row below the
// board, and the reference's legal_actions / apply_action raise IndexError on
// every call (boardConfig.py:27,45-59; boardv2.py:188 calls legal_actions in
// every step). Such a BoardConfig resets (BoardV2.__init__) but cannot step.
int check_ids_on_board(const m3_ctx* c) {
    if (c->R >= c->C) return M3_OK;
    return set_err(M3_ERR_INVALID,
                   "BoardConfig(rows=%d, columns=%d): action ids reach row %d, past the board; the reference's "
                   "legal_actions / apply_action raise IndexError for rows < columns", c->R, c->C, c->R);
}

int ensure_scratch(m3_ctx* c, size_t bytes) {
    if (c->dcap >= bytes) return M3_OK;
    HIP_TRY(hipStreamSynchronize(c->stream));  // async work may still use the old buffer
    if (c->dbuf) HIP_TRY(hipFree(c->dbuf));
    c->dbuf = nullptr;
    c->dcap = 0;
    HIP_TRY(hipMalloc(&c->dbuf, bytes));
    c->dcap = bytes;
    return M3_OK;
}

struct Carve {
    char* base;
    size_t off = 0;
    template <class T>
    T* take(size_t count) {
        off = (off + 255) & ~size_t(255);
        T* p = reinterpret_cast<T*>(base + off);
        off += count * sizeof(T);
        return p;
    }
};

size_t carve_size(std::initializer_list<size_t> sizes) {
    size_t s = 0;
    for (size_t v : sizes) s = ((s + 255) & ~size_t(255)) + v;
    return s + 256;
}

// Host-buffer calls stage through one pinned image per direction: the caller's
// inputs are packed into the context's pinned buffer and go up in ONE copy
// (which also zeroes the launch's counters, part of the image), the outputs
// come back in ONE copy and are unpacked -- for the BoardV2 facade's batch-1
// calls that is two copies, the launches and a sync, instead of a pageable
// copy per array.
struct Image {
    static constexpr int MAXP = 12;
    size_t off[MAXP] = {}, size[MAXP] = {};
    int n = 0;
    size_t total = 0;
    int add(size_t bytes) {
        total = (total + 255) & ~size_t(255);
        off[n] = total;
        size[n] = bytes;
        total += bytes;
        return n++;
    }
};

int ensure_host(m3_ctx* c, size_t bytes) {
    if (c->hcap >= bytes) return M3_OK;
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (c->hbuf) HIP_TRY(hipHostFree(c->hbuf));
    c->hbuf = nullptr;
    c->hdev = nullptr;
    c->hcap = 0;
    HIP_TRY(hipHostMalloc(&c->hbuf, bytes, hipHostMallocMapped | hipHostMallocPortable));
    HIP_TRY(hipHostGetDevicePointer(&c->hdev, c->hbuf, 0));  // the device's address of the same bytes
    c->hcap = bytes;
    return M3_OK;
}

// Device scratch = [input image | output image | device-only tail]; the pinned
// buffer holds the larger of the two images. Returns the device base.
int stage_begin(m3_ctx* c, const Image& in, const Image& out, size_t tail, char** dev) {
    const size_t in_sz = (in.total + 255) & ~size_t(255), out_sz = (out.total + 255) & ~size_t(255);
    int rc = ensure_scratch(c, in_sz + out_sz + tail + 256);
    if (rc) return rc;
    rc = ensure_host(c, std::max(in_sz, out_sz) + 256);
    if (rc) return rc;
    *dev = (char*)c->dbuf;
    return M3_OK;
}

// pack host inputs and upload the image; the same copy zeroes the first
// `zero_out` bytes of the output image that follows it (the launch's counters)
int stage_upload(m3_ctx* c, const Image& in, std::initializer_list<const void*> srcs, char* dev,
                 size_t zero_out = 0) {
    char* h = (char*)c->hbuf;
    int i = 0;
    for (const void* p : srcs) {
        memcpy(h + in.off[i], p, in.size[i]);
        ++i;
    }
    const size_t in_sz = (in.total + 255) & ~size_t(255);
    memset(h + in.total, 0, in_sz + zero_out - in.total);
    HIP_TRY(hipMemcpyAsync(dev, h, in_sz + zero_out, hipMemcpyHostToDevice, c->stream));
    return M3_OK;
}

// download the output image, wait, unpack into the caller's buffers (nullptr = skip)
int stage_download(m3_ctx* c, const Image& out, std::initializer_list<void*> dsts, const char* dev) {
    char* h = (char*)c->hbuf;
    HIP_TRY(hipMemcpyAsync(h, dev, out.total, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    int i = 0;
    for (void* p : dsts) {
        if (p) memcpy(p, h + out.off[i], out.size[i]);
        ++i;
    }
    return M3_OK;
}

int bad_cells_error() {
    return set_err(M3_ERR_INVALID, "cell value outside [0, 127] in the boards (outputs undefined)");
}

// Zero-copy path of the small host-buffer calls (the facade's batch-1 calls): the kernels read
// the inputs from and write the outputs to the context's pinned buffer (host memory the device
// maps), so a call is its launches and one sync, with no copy in either direction.
constexpr int64_t ZC_MAX_BOARDS = 256;
constexpr int ZC_OVF_WORD = 8;  // c->counters[8]: the zero-copy overflow count, kept zero between calls








// Make `st` wait for every shard's last enqueued work.
int join_shards(m3_env* e, hipStream_t st) {
    for (auto& sh : e->shards)
        if (sh.n) HIP_TRY(hipStreamWaitEvent(st, sh.ev, 0));
    return M3_OK;
}

int sync_env(m3_env* e) {
    for (auto& sh : e->shards) {
        HIP_TRY(hipStreamSynchronize(sh.stream));
        HIP_TRY(hipStreamSynchronize(sh.pstream));
        for (bool& p : sh.ppending) p = false;
        for (bool& p : sh.apending) p = false;
    }
    if (e->ustream) HIP_TRY(hipStreamSynchronize(e->ustream));
    e->upload_pend[0] = e->upload_pend[1] = false;
    HIP_TRY(hipStreamSynchronize(e->ctx->stream));
    return M3_OK;
}

void destroy_shards(m3_env* e) {
    for (auto& sh : e->shards) {
        (void)hipStreamDestroy(sh.stream);
        (void)hipStreamDestroy(sh.pstream);
        (void)hipEventDestroy(sh.ev);
        for (hipEvent_t ev : sh.pev) (void)hipEventDestroy(ev);
        for (hipEvent_t ev : sh.aev) (void)hipEventDestroy(ev);
    }
    e->shards.clear();
}
}  // namespace

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
// configuration id (shape_id) -> its config type (CF_<id>, m3_kernels.hpp)
template <class F>
static int with_shape(int shape, F&& f) {
    static_assert(N_CONFIGS == 10, "with_shape lists every configuration");
    switch (shape) {
        case 0: return f(CF_0{});
        case 1: return f(CF_1{});
#ifndef M3_HEADLINE_ONLY
        case 2: return f(CF_2{});
        case 3: return f(CF_3{});
        case 4: return f(CF_4{});
        case 5: return f(CF_5{});
#ifndef M3_NO_WIDE_FRAME
        case 6: return f(CF_6{});
        case 7: return f(CF_7{});
        case 8: return f(CF_8{});
        case 9: return f(CF_9{});
#endif
#endif
        default: return set_err(M3_ERR_UNSUPPORTED, "board shape not compiled in");
    }
}

static int ensure_fresh(m3_env* e) {
    if (!e->stale) return M3_OK;
    return with_shape(e->ctx->shape, [&](auto cf) { return rederive<decltype(cf)>(e); });
}

extern "C" {

int m3_abi_version(void) { return M3_ABI_VERSION; }

const char* m3_last_error(void) { return g_err.c_str(); }

int m3_device_count(int* out) {
    CHECK_ARG(out, "null out");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    *out = (e == hipSuccess) ? n : 0;
    return M3_OK;
}

int m3_supported(int rows, int columns, int types) { return shape_id(rows, columns, types) >= 0 ? 1 : 0; }

int m3_action_space(int rows, int columns, int* out_actions, int* out_words) {
    CHECK_ARG(rows > 0 && columns > 0, "bad shape");
    const int A = rows * (columns - 1) * 2;
    if (out_actions) *out_actions = A;
    if (out_words) *out_words = (A + 31) / 32;
    return M3_OK;
}

int m3_ctx_create(int device, int rows, int columns, int types, m3_ctx** out) {
    CHECK_ARG(out, "null out");
    *out = nullptr;
    const int sid = shape_id(rows, columns, types);
    if (sid < 0)
        return set_err(M3_ERR_UNSUPPORTED,
                       "BoardConfig(rows=%d, columns=%d, types=%d): supported are rows and columns 3..32, "
                       "types 2..31", rows, columns, types);
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return set_err(M3_ERR_NO_DEVICE, "no HIP device visible (libm3 has no CPU fallback)");
    CHECK_ARG(device >= 0 && device < ndev, "device index out of range");
    HIP_TRY(hipSetDevice(device));
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, device));
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return set_err(M3_ERR_NO_DEVICE, "device %d is %s; libm3 is built for gfx950 only", device, prop.gcnArchName);
    m3_ctx* c = new m3_ctx;
    c->device = device;
    c->R = rows;
    c->C = columns;
    c->T = types;
    c->N = rows * columns;
    c->A = rows * (columns - 1) * 2;
    c->AW = (c->A + 31) / 32;
    c->shape = sid;
    c->sdesc = make_shape(rows, columns, types);
    hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipMalloc(&c->counters, 256);
    if (e == hipSuccess) e = hipMemset(c->counters, 0, 256);  // (the zero-copy overflow word starts at zero)
    if (e != hipSuccess) {
        delete c;
        return set_err(M3_ERR_HIP, "context setup: %s", hipGetErrorString(e));
    }
    *out = c;
    return M3_OK;
}

int m3_ctx_destroy(m3_ctx* c) {
    if (!c) return M3_OK;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->dbuf) (void)hipFree(c->dbuf);
    if (c->hbuf) (void)hipHostFree(c->hbuf);
    if (c->counters) (void)hipFree(c->counters);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
    return M3_OK;
}

int m3_ctx_synchronize(m3_ctx* c) {
    CHECK_ARG(c, "null ctx");
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return M3_OK;
}

int m3_dev_alloc(m3_ctx* c, int64_t bytes, void** out) {
    CHECK_ARG(c && out && bytes >= 0, "bad arguments");
    *out = nullptr;
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipMalloc(out, bytes ? (size_t)bytes : 4));
    return M3_OK;
}

int m3_dev_free(m3_ctx* c, void* p) {
    CHECK_ARG(c, "null ctx");
    if (!p) return M3_OK;
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipStreamSynchronize(c->stream));  // the context's work may still use it
    HIP_TRY(hipFree(p));
    return M3_OK;
}

int m3_dev_copy(m3_ctx* c, void* dst, const void* src, int64_t bytes, int kind) {
    CHECK_ARG(c && dst && src && bytes >= 0 && (kind == 1 || kind == 2), "bad arguments");
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipMemcpyAsync(dst, src, (size_t)bytes, kind == 1 ? hipMemcpyHostToDevice : hipMemcpyDeviceToHost,
                           c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return M3_OK;
}

int m3_init_boards_ex(m3_ctx* c, int64_t n, const uint32_t* seeds, int8_t* out_boards, uint32_t* out_draws,
                      int32_t* out_first_action, uint32_t* out_flags) {
    CHECK_ARG(c && n >= 0 && (n == 0 || (seeds && out_boards)), "bad arguments");
    if (n == 0) return M3_OK;
    HIP_TRY(hipSetDevice(c->device));
    if (n <= ZC_MAX_BOARDS) {  // zero-copy: the reset launch(es) and one sync
        Image im;
        const int i_s = im.add(n * 4ull), o_b = im.add(n * (size_t)c->N), o_d = im.add(n * 4ull),
                  o_f = im.add(n * 4ull), o_g = im.add(n * 4ull);
        int rc = ensure_host(c, im.total + 256);
        if (rc) return rc;
        char* h = (char*)c->hbuf;
        char* d = (char*)c->hdev;
        memcpy(h + im.off[i_s], seeds, n * 4);
        InitArgs a{};
        a.shape = c->sdesc;
        a.n = n;
        a.seeds = (const uint32_t*)(d + im.off[i_s]);
        a.boards = (int8_t*)(d + im.off[o_b]);
        a.draws = (uint32_t*)(d + im.off[o_d]);
        a.first_action = (int32_t*)(d + im.off[o_f]);
        a.flags = (uint32_t*)(d + im.off[o_g]);
        rc = with_shape(c->shape, [&](auto cf) { return launch_init<decltype(cf)>(c->stream, a, n); });
        if (rc) return rc;
        HIP_TRY(hipStreamSynchronize(c->stream));
        memcpy(out_boards, h + im.off[o_b], n * (size_t)c->N);
        if (out_draws) memcpy(out_draws, h + im.off[o_d], n * 4);
        if (out_first_action) memcpy(out_first_action, h + im.off[o_f], n * 4);
        if (out_flags) memcpy(out_flags, h + im.off[o_g], n * 4);
        return M3_OK;
    }
    Image in, out;
    in.add(n * 4ull);
    const int o_b = out.add(n * (size_t)c->N), o_d = out.add(n * 4ull), o_f = out.add(n * 4ull),
              o_g = out.add(n * 4ull);
    char* dev;
    int rc = stage_begin(c, in, out, 0, &dev);
    if (rc) return rc;
    char* dout = dev + ((in.total + 255) & ~size_t(255));
    rc = stage_upload(c, in, {seeds}, dev);
    if (rc) return rc;
    InitArgs a{};
    a.shape = c->sdesc;
    a.n = n;
    a.seeds = (const uint32_t*)dev;
    a.boards = (int8_t*)(dout + out.off[o_b]);
    a.draws = (uint32_t*)(dout + out.off[o_d]);
    a.first_action = (int32_t*)(dout + out.off[o_f]);
    a.flags = (uint32_t*)(dout + out.off[o_g]);
    rc = with_shape(c->shape, [&](auto cf) { return launch_init<decltype(cf)>(c->stream, a, n); });
    if (rc) return rc;
    return stage_download(c, out, {out_boards, out_draws, out_first_action, out_flags}, dout);
}

int m3_init_boards(m3_ctx* c, int64_t n, const uint32_t* seeds, int8_t* out_boards, uint32_t* out_draws,
                   int32_t* out_first_action) {
    std::vector<uint32_t> flags(n > 0 ? (size_t)n : 0);
    int rc = m3_init_boards_ex(c, n, seeds, out_boards, out_draws, out_first_action, flags.data());
    if (rc) return rc;
    int64_t capped = 0;
    for (uint32_t f : flags) capped += (f & M3_FLAG_RESET_CAP) != 0;
    if (capped)  // the reference keeps drawing (boardv2.py:23-27): no result to return
        return set_err(M3_ERR_CAP, "%lld of %lld resets stopped at the redraw-round cap (M3_FLAG_RESET_CAP; "
                       "m3_init_boards_ex returns the flags per board)", (long long)capped, (long long)n);
    return M3_OK;
}

int m3_apply_actions(m3_ctx* c, int64_t n, const int8_t* boards, const uint32_t* seeds, const int32_t* n_actions,
                     const int32_t* actions, int8_t* out_boards, int32_t* out_reward, uint32_t* out_draws,
                     uint32_t* out_flags, uint32_t* out_legal_bits, int32_t* out_next_action) {
    CHECK_ARG(c && n >= 0, "bad arguments");
    if (n == 0) return M3_OK;
    CHECK_ARG(boards && seeds && n_actions && actions && out_boards && out_reward && out_draws && out_flags,
              "null buffer");
    int rc0 = check_ids_on_board(c);
    if (rc0) return rc0;
    HIP_TRY(hipSetDevice(c->device));
    const size_t bytes = n * (size_t)c->N;
    if (n <= ZC_MAX_BOARDS) {  // zero-copy: two launches and one sync
        Image im;
        const int i_b = im.add(bytes), i_s = im.add(n * 4ull), i_na = im.add(n * 4ull), i_a = im.add(n * 4ull);
        const int o_bad = im.add(16), o_b = im.add(bytes), o_r = im.add(n * 4ull), o_d = im.add(n * 4ull),
                  o_f = im.add(n * 4ull), o_l = im.add(out_legal_bits ? n * 4ull * c->AW : 0),
                  o_x = im.add(out_next_action ? n * 4ull : 0);
        int rc = ensure_host(c, im.total + 256);
        if (rc) return rc;
        rc = ensure_scratch(c, n * 4ull + 256);
        if (rc) return rc;
        char* h = (char*)c->hbuf;  // host view
        char* d = (char*)c->hdev;  // device view of the same pinned bytes
        memcpy(h + im.off[i_b], boards, bytes);
        memcpy(h + im.off[i_s], seeds, n * 4);
        memcpy(h + im.off[i_na], n_actions, n * 4);
        memcpy(h + im.off[i_a], actions, n * 4);
        memset(h + im.off[o_bad], 0, 16);
        ApplyArgs a{};
        a.shape = c->sdesc;
        a.n = n;
        a.boards = (const int8_t*)(d + im.off[i_b]);
        a.seeds = (const uint32_t*)(d + im.off[i_s]);
        a.n_actions = (const int32_t*)(d + im.off[i_na]);
        a.actions = (const int32_t*)(d + im.off[i_a]);
        a.out_boards = (int8_t*)(d + im.off[o_b]);
        a.reward = (int32_t*)(d + im.off[o_r]);
        a.draws = (uint32_t*)(d + im.off[o_d]);
        a.flags = (uint32_t*)(d + im.off[o_f]);
        a.legal = out_legal_bits ? (uint32_t*)(d + im.off[o_l]) : nullptr;
        a.next_action = out_next_action ? (int32_t*)(d + im.off[o_x]) : nullptr;
        a.ovf_count = c->counters + ZC_OVF_WORD;
        a.bad_cells = (uint32_t*)(d + im.off[o_bad]);
        a.ovf_list = (uint32_t*)c->dbuf;
        a.clear_ovf = 1;
        rc = with_shape(c->shape, [&](auto cf) { return launch_apply<decltype(cf)>(c, a); });
        if (rc) {  // k_apply may have counted overflows that k_apply_fix never cleared: the next
                   // call must not read them (best effort; the launch error is what is reported)
            (void)hipStreamSynchronize(c->stream);
            (void)hipMemset(a.ovf_count, 0, 4);
            return rc;
        }
        HIP_TRY(hipStreamSynchronize(c->stream));
        if (*(volatile uint32_t*)(h + im.off[o_bad])) return bad_cells_error();
        memcpy(out_boards, h + im.off[o_b], bytes);
        memcpy(out_reward, h + im.off[o_r], n * 4);
        memcpy(out_draws, h + im.off[o_d], n * 4);
        memcpy(out_flags, h + im.off[o_f], n * 4);
        if (out_legal_bits) memcpy(out_legal_bits, h + im.off[o_l], n * 4ull * c->AW);
        if (out_next_action) memcpy(out_next_action, h + im.off[o_x], n * 4);
        return M3_OK;
    }
    Image in, out;  // cell values are checked on the device while the boards are staged (k_apply)
    const int i_b = in.add(bytes), i_s = in.add(n * 4ull), i_na = in.add(n * 4ull), i_a = in.add(n * 4ull);
    const int o_cnt = out.add(16), o_b = out.add(bytes), o_r = out.add(n * 4ull), o_d = out.add(n * 4ull),
              o_f = out.add(n * 4ull), o_l = out.add(out_legal_bits ? n * 4ull * c->AW : 0),
              o_x = out.add(out_next_action ? n * 4ull : 0);
    char* dev;
    int rc = stage_begin(c, in, out, n * 4ull, &dev);
    if (rc) return rc;
    char* dout = dev + ((in.total + 255) & ~size_t(255));
    char* dtail = dout + ((out.total + 255) & ~size_t(255));
    rc = stage_upload(c, in, {boards, seeds, n_actions, actions}, dev, 16);
    if (rc) return rc;
    ApplyArgs a{};
    a.shape = c->sdesc;
    a.n = n;
    a.boards = (const int8_t*)(dev + in.off[i_b]);
    a.seeds = (const uint32_t*)(dev + in.off[i_s]);
    a.n_actions = (const int32_t*)(dev + in.off[i_na]);
    a.actions = (const int32_t*)(dev + in.off[i_a]);
    a.out_boards = (int8_t*)(dout + out.off[o_b]);
    a.reward = (int32_t*)(dout + out.off[o_r]);
    a.draws = (uint32_t*)(dout + out.off[o_d]);
    a.flags = (uint32_t*)(dout + out.off[o_f]);
    a.legal = out_legal_bits ? (uint32_t*)(dout + out.off[o_l]) : nullptr;
    a.next_action = out_next_action ? (int32_t*)(dout + out.off[o_x]) : nullptr;
    a.ovf_count = (uint32_t*)(dout + out.off[o_cnt]);  // zeroed by the upload, returned with the outputs
    a.bad_cells = a.ovf_count + 1;
    a.ovf_list = (uint32_t*)dtail;
    rc = with_shape(c->shape, [&](auto cf) { return launch_apply<decltype(cf)>(c, a); });
    if (rc) return rc;
    uint32_t cnt[4];
    rc = stage_download(c, out, {cnt, out_boards, out_reward, out_draws, out_flags, out_legal_bits,
                                 out_next_action}, dout);
    if (rc) return rc;
    return cnt[1] ? bad_cells_error() : M3_OK;
}

int m3_legal_actions(m3_ctx* c, int64_t n, const int8_t* boards, uint32_t* out_legal_bits) {
    CHECK_ARG(c && n >= 0, "bad arguments");
    if (n == 0) return M3_OK;
    CHECK_ARG(boards && out_legal_bits, "null buffer");
    int rc0 = check_ids_on_board(c);
    if (rc0) return rc0;
    HIP_TRY(hipSetDevice(c->device));
    if (n <= ZC_MAX_BOARDS) {  // zero-copy: one launch and one sync
        Image im;
        const int i_b = im.add(n * (size_t)c->N), o_l = im.add(n * 4ull * c->AW);
        int rc = ensure_host(c, im.total + 256);
        if (rc) return rc;
        char* h = (char*)c->hbuf;
        char* d = (char*)c->hdev;
        memcpy(h + im.off[i_b], boards, n * (size_t)c->N);
        rc = with_shape(c->shape, [&](auto cf) {
            return launch_legal<decltype(cf)>(c, n, (const int8_t*)(d + im.off[i_b]), (uint32_t*)(d + im.off[o_l]));
        });
        if (rc) return rc;
        HIP_TRY(hipStreamSynchronize(c->stream));
        memcpy(out_legal_bits, h + im.off[o_l], n * 4ull * c->AW);
        return M3_OK;
    }
    Image in, out;
    in.add(n * (size_t)c->N);
    out.add(n * 4ull * c->AW);
    char* dev;
    int rc = stage_begin(c, in, out, 0, &dev);
    if (rc) return rc;
    char* dout = dev + ((in.total + 255) & ~size_t(255));
    rc = stage_upload(c, in, {boards}, dev);
    if (rc) return rc;
    rc = with_shape(c->shape, [&](auto cf) {
        return launch_legal<decltype(cf)>(c, n, (const int8_t*)dev, (uint32_t*)dout);
    });
    if (rc) return rc;
    return stage_download(c, out, {out_legal_bits}, dout);
}

// ---- rollouts ---------------------------------------------------------------
}  // extern "C"

namespace {

// overflow list + group-table spill pool of a rollout launch (a lane keeps one
// spill record for its whole rollout)
// records of the rollout spill pool: one per 8 rollouts (at least 4096), within 256 MB (a lane
// that finds the pool empty is replayed exactly by k_rollout_fix)
int64_t rollout_spill_cap(int64_t n, size_t words) {
    const int64_t budget = (int64_t)((256ull << 20) / (words * 4ull));
    return std::max<int64_t>(1, std::min(std::max<int64_t>(4096, n / 8), budget));
}

size_t rollout_spill_words(int shape) {
    return (size_t)with_shape(shape, [&](auto cf) {
        using CF = decltype(cf);
        return (int)LdsStore<CF, KS<CF>::GCAP, KS<CF>::B>::SPILL_WORDS;
    });
}

// a.n and the per-rollout buffers set; carves the pool from cv and launches.
// counters: 16 zeroed bytes on the device (nullptr: the context's, zeroed here)
int enqueue_rollouts(m3_ctx* c, RolloutArgs a, Carve& cv, uint32_t* counters = nullptr) {
    const int64_t cap = rollout_spill_cap(a.n, rollout_spill_words(c->shape));
    if (!counters) {
        counters = c->counters;
        HIP_TRY(hipMemsetAsync(counters, 0, 16, c->stream));
    }
    a.counters = counters;
    a.ovf_list = cv.take<uint32_t>(a.n);
    a.spill = cv.take<uint32_t>(cap * rollout_spill_words(c->shape));
    a.spill_cap = (uint32_t)cap;
    return with_shape(c->shape, [&](auto cf) { return launch_rollouts<decltype(cf)>(c, a); });
}

}  // namespace

extern "C" {

int m3_rollouts_device(m3_ctx* c, int64_t n, const int8_t* boards, const uint32_t* seeds, const int32_t* n_actions,
                       const uint32_t* rollout_seeds, int32_t* out_gain, int32_t* out_steps, uint32_t* out_draws,
                       uint32_t* out_flags, int8_t* out_boards) {
    CHECK_ARG(c && n >= 0, "bad arguments");
    if (n == 0) return M3_OK;
    CHECK_ARG(n < (int64_t)1 << 31, "n too large");
    CHECK_ARG(boards && seeds && n_actions && rollout_seeds && out_gain && out_steps && out_draws && out_flags,
              "null buffer");
    int rc0 = check_ids_on_board(c);
    if (rc0) return rc0;
    HIP_TRY(hipSetDevice(c->device));
    int rc = ensure_scratch(c, carve_size({n * 4ull, rollout_spill_cap(n, rollout_spill_words(c->shape)) * rollout_spill_words(c->shape) * 4ull}));
    if (rc) return rc;
    Carve cv{(char*)c->dbuf};
    RolloutArgs a{};
    a.shape = c->sdesc;
    a.n = n;
    a.boards = boards;
    a.seeds = seeds;
    a.n_actions = n_actions;
    a.rseeds = rollout_seeds;
    a.gain = out_gain;
    a.steps = out_steps;
    a.draws = out_draws;
    a.flags = out_flags;
    a.out_boards = out_boards;
    return enqueue_rollouts(c, a, cv);
}

int m3_rollouts(m3_ctx* c, int64_t n, const int8_t* boards, const uint32_t* seeds, const int32_t* n_actions,
                const uint32_t* rollout_seeds, int32_t* out_gain, int32_t* out_steps, uint32_t* out_draws,
                uint32_t* out_flags, int8_t* out_boards) {
    CHECK_ARG(c && n >= 0, "bad arguments");
    if (n == 0) return M3_OK;
    CHECK_ARG(n < (int64_t)1 << 31, "n too large");
    CHECK_ARG(boards && seeds && n_actions && rollout_seeds && out_gain && out_steps && out_draws && out_flags,
              "null buffer");
    int rc0 = check_ids_on_board(c);
    if (rc0) return rc0;
    HIP_TRY(hipSetDevice(c->device));
    const size_t bytes = n * (size_t)c->N;
    Image in, out;  // cell values are checked on the device while the boards are staged (k_rollout)
    const int i_b = in.add(bytes), i_s = in.add(n * 4ull), i_na = in.add(n * 4ull), i_rs = in.add(n * 4ull);
    const int o_cnt = out.add(16), o_g = out.add(n * 4ull), o_st = out.add(n * 4ull), o_d = out.add(n * 4ull),
              o_f = out.add(n * 4ull), o_b = out.add(out_boards ? bytes : 0);
    const size_t tail = carve_size({n * 4ull, rollout_spill_cap(n, rollout_spill_words(c->shape)) * rollout_spill_words(c->shape) * 4ull});
    char* dev;
    int rc = stage_begin(c, in, out, tail, &dev);
    if (rc) return rc;
    char* dout = dev + ((in.total + 255) & ~size_t(255));
    char* dtail = dout + ((out.total + 255) & ~size_t(255));
    rc = stage_upload(c, in, {boards, seeds, n_actions, rollout_seeds}, dev, 16);
    if (rc) return rc;
    RolloutArgs a{};
    a.shape = c->sdesc;
    a.n = n;
    a.boards = (const int8_t*)(dev + in.off[i_b]);
    a.seeds = (const uint32_t*)(dev + in.off[i_s]);
    a.n_actions = (const int32_t*)(dev + in.off[i_na]);
    a.rseeds = (const uint32_t*)(dev + in.off[i_rs]);
    a.gain = (int32_t*)(dout + out.off[o_g]);
    a.steps = (int32_t*)(dout + out.off[o_st]);
    a.draws = (uint32_t*)(dout + out.off[o_d]);
    a.flags = (uint32_t*)(dout + out.off[o_f]);
    a.out_boards = out_boards ? (int8_t*)(dout + out.off[o_b]) : nullptr;
    Carve cv{dtail};
    rc = enqueue_rollouts(c, a, cv, (uint32_t*)(dout + out.off[o_cnt]));  // zeroed by the upload
    if (rc) return rc;
    uint32_t cnt[4];
    rc = stage_download(c, out, {cnt, out_gain, out_steps, out_draws, out_flags, out_boards}, dout);
    if (rc) return rc;
    return cnt[2] ? bad_cells_error() : M3_OK;
}

// ---- env ------------------------------------------------------------------
int m3_env_create(m3_ctx* c, int64_t n, int num_moves, int env_goal, m3_env** out) {
    CHECK_ARG(c && out && n > 0 && num_moves > 0, "bad arguments");
    CHECK_ARG(n < (int64_t)1 << 31, "n too large");
    int rc0 = check_ids_on_board(c);
    if (rc0) return rc0;
    *out = nullptr;
    HIP_TRY(hipSetDevice(c->device));
    m3_env* e = new m3_env;
    e->ctx = c;
    e->n = n;
    e->num_moves = num_moves;
    e->goal = env_goal;
    const size_t bytes = n * (size_t)c->N;
    hipError_t err = hipSuccess;
    auto alloc = [&](auto** p, size_t sz) {
        if (err == hipSuccess) err = hipMalloc((void**)p, sz ? sz : 4);
    };
    alloc(&e->boards[0], bytes);
    alloc(&e->boards[1], bytes);
    alloc(&e->seeds, n * 4);
    alloc(&e->flags, n * 4);
    alloc(&e->draws, n * 4);
    alloc(&e->legal, n * 4ull * c->AW);
    alloc(&e->score, n * 4);
    alloc(&e->moves, n * 4);
    alloc(&e->next_action, n * 4);
    alloc(&e->reward, n * 4);
    alloc(&e->done, n);
    alloc(&e->trunc, n);
    alloc(&e->counters, 64 * 4 * MAX_SHARDS);
    alloc(&e->ovf_list, n * 4);
    alloc(&e->packed, 2 * n * 4);
    alloc(&e->slot, n);
    alloc(&e->ne_words, (size_t)NSLOT * n * 4ull * ((c->N + 3) / 4));
    alloc(&e->ne_first, (size_t)NSLOT * n * 4);
    alloc(&e->ne_legal, (size_t)NSLOT * n * 4ull * c->AW);
    alloc(&e->ne_flags, (size_t)NSLOT * n * 4);
    alloc(&e->defer, n * 4);
    for (int p = 0; p < PF_LAG; ++p) {
        alloc(&e->pf_list[p], n * 4);
        alloc(&e->pf_seed[p], n * 4);
        alloc(&e->pf_slot[p], n * 4);
    }
    with_shape(c->shape, [&](auto cf) {
        using K = KS<decltype(cf)>;
        using St = LdsStore<decltype(cf), K::GCAP, K::B>;
        alloc(&e->spill, (size_t)MAX_SHARDS * K::SPILL_RECORDS * St::SPILL_WORDS * 4);
        alloc(&e->m397, (size_t)NSLOT * n * 4ull);
        constexpr size_t RW = CONT_REC<decltype(cf)>;
        if constexpr (K::CASCADE_LIMIT >= 0) alloc(&e->cont, RW * n * 4ull);
        if constexpr (RESET_TWO_STAGE<decltype(cf)>) alloc(&e->tab, (size_t)TwoStage<decltype(cf)>::TW * n * 4ull);
        if constexpr (RESET_TWO_STAGE_REJ<decltype(cf)>)
            alloc(&e->tab, (size_t)TwoStageRej<decltype(cf)>::TW * n * 4ull);
        return 0;
    });
    for (hipEvent_t& ev : e->gev)
        if (err == hipSuccess) err = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    // every per-board field starts zeroed: a never-reset env reads back zeros, not stale device memory
    {
        void* zp[] = {e->boards[0], e->boards[1], e->seeds, e->flags, e->draws, e->legal, e->score, e->moves,
                      e->next_action, e->reward, e->done, e->trunc, e->slot};
        size_t zb[] = {bytes, bytes, n * 4ull, n * 4ull, n * 4ull, n * 4ull * c->AW, n * 4ull, n * 4ull,
                       n * 4ull, n * 4ull, (size_t)n, (size_t)n, (size_t)n};
        for (int i = 0; i < 13 && err == hipSuccess; ++i) err = hipMemset(zp[i], 0, zb[i]);
    }
    if (err != hipSuccess) {
        m3_env_destroy(e);
        return set_err(M3_ERR_HIP, "env allocation (%lld boards): %s", (long long)n, hipGetErrorString(err));
    }
    // default: one shard. Every shard adds two streams (step + prefetch), and
    // streams beyond GPU_MAX_HW_QUEUES (HIP default 4) share hardware queues,
    // so a step queues behind a reset launch. Measured at 1,048,576 boards
    // (9x9x6, autoreset, gpurun_out/q1-q3): 4 queues: 1 / 2 / 4 shards = 1.75 /
    // 1.43 / 1.18 G env-steps/s; 8 queues: 1.74 / 1.98 / 1.38 (2 shards fill
    // each other's kernel tails); one prefetch stream shared by 2 shards: 1.67.
    int rc = m3_env_set_shards(e, 1);
    if (rc) {
        m3_env_destroy(e);
        return rc;
    }
    *out = e;
    return M3_OK;
}

int m3_env_set_shards(m3_env* e, int nshards) {
    CHECK_ARG(e && nshards >= 1 && nshards <= MAX_SHARDS, "nshards must be in [1, 8]");
    HIP_TRY(hipSetDevice(e->ctx->device));
    int rc = sync_env(e);
    if (rc) return rc;
    destroy_shards(e);
    // shard boundaries on 256-board multiples
    const int64_t per = ((e->n + nshards - 1) / nshards + BLOCK - 1) / BLOCK * BLOCK;
    for (int s = 0; s < nshards; ++s) {
        m3_env::Shard sh;
        sh.off = std::min<int64_t>(e->n, s * per);
        sh.n = std::min<int64_t>(e->n, sh.off + per) - sh.off;
        if (M3_STREAM_PRIO) {  // the step stream first at dispatch, the prefetch resets last
            int least = 0, greatest = 0;
            HIP_TRY(hipDeviceGetStreamPriorityRange(&least, &greatest));
            HIP_TRY(hipStreamCreateWithPriority(&sh.stream, hipStreamNonBlocking, greatest));
            HIP_TRY(hipStreamCreateWithPriority(&sh.pstream, hipStreamNonBlocking, least));
        } else {
            HIP_TRY(hipStreamCreateWithFlags(&sh.stream, hipStreamNonBlocking));
            HIP_TRY(hipStreamCreateWithFlags(&sh.pstream, hipStreamNonBlocking));
        }
        HIP_TRY(hipEventCreateWithFlags(&sh.ev, hipEventDisableTiming));
        for (hipEvent_t& ev : sh.pev) HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        for (hipEvent_t& ev : sh.aev) HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        e->shards.push_back(sh);
    }
    return M3_OK;
}

int m3_env_synchronize(m3_env* e) {
    CHECK_ARG(e, "null env");
    HIP_TRY(hipSetDevice(e->ctx->device));
    int rc = sync_env(e);
    if (rc) return rc;
    return ensure_fresh(e);
}

int m3_env_destroy(m3_env* e) {
    if (!e) return M3_OK;
    (void)hipSetDevice(e->ctx->device);
    (void)sync_env(e);
    destroy_shards(e);
    for (int p = 0; p < 2; ++p) {
        if (e->upload_ev[p]) (void)hipEventDestroy(e->upload_ev[p]);
        if (e->hstage[p]) (void)hipHostFree(e->hstage[p]);
    }
    if (e->ustream) (void)hipStreamDestroy(e->ustream);
    for (hipEvent_t ev : e->gev)
        if (ev) (void)hipEventDestroy(ev);
    void* ptrs[] = {e->boards[0], e->boards[1], e->seeds, e->flags, e->draws, e->legal, e->score, e->moves,
                    e->next_action, e->reward, e->done, e->trunc, e->actions[0], e->actions[1], e->counters,
                    e->ovf_list,
                    e->packed, e->gathered, e->slot, e->ne_words, e->ne_first, e->ne_legal, e->ne_flags,
                    e->spill, e->m397, e->cont, e->defer, e->tab};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    for (int q = 0; q < PF_LAG; ++q)
        for (void* p : {(void*)e->pf_list[q], (void*)e->pf_seed[q], (void*)e->pf_slot[q]})
            if (p) (void)hipFree(p);
    if (e->comm) ncclCommDestroy(e->comm);
    for (hipEvent_t ev : e->tev) (void)hipEventDestroy(ev);
    delete e;
    return M3_OK;
}

int m3_env_reset(m3_env* e, const uint32_t* seeds, uint32_t seed_base) {
    CHECK_ARG(e, "null env");
    m3_ctx* c = e->ctx;
    HIP_TRY(hipSetDevice(c->device));
    int rc0 = sync_env(e);
    if (rc0) return rc0;
    if (seeds) {
        HIP_TRY(hipMemcpyAsync(e->seeds, seeds, e->n * 4, hipMemcpyHostToDevice, c->stream));
    } else {
        // seeds = seed_base + i, written on host once (reset is not on the hot path)
        uint32_t* h = (uint32_t*)malloc(e->n * 4);
        if (!h) return set_err(M3_ERR_INVALID, "host allocation failed");
        for (int64_t i = 0; i < e->n; ++i) h[i] = seed_base + (uint32_t)i;
        hipError_t err = hipMemcpy(e->seeds, h, e->n * 4, hipMemcpyHostToDevice);
        free(h);
        HIP_TRY(err);
    }
    InitArgs a{};
    a.shape = c->sdesc;
    a.n = e->n;
    a.seeds = e->seeds;
    a.boards = e->boards[e->cur];
    a.first_action = e->next_action;
    a.legal = e->legal;
    a.score = e->score;
    a.moves = e->moves;
    a.reward = e->reward;
    a.done = e->done;
    a.trunc = e->trunc;
    a.flags = e->flags;
    a.draws = e->draws;
    a.m397 = e->m397;
    a.cstride = e->n;
    HIP_TRY(hipMemsetAsync(e->counters, 0, 64 * 4 * MAX_SHARDS, c->stream));  // also clears the stats
    HIP_TRY(hipMemsetAsync(e->slot, 0, e->n, c->stream));
    e->steps = 0;
    int rc = with_shape(c->shape, [&](auto cf) {
        int r = launch_init<decltype(cf)>(c->stream, a, e->n);
        if (r == M3_OK && e->autoreset) r = fill_next_slots<decltype(cf)>(e);
        return r;
    });
    if (rc) return rc;
    HIP_TRY(hipStreamSynchronize(c->stream));
    e->ready = true;
    e->stale = false;
    return M3_OK;
}

int m3_env_set_autoreset(m3_env* e, int enabled, uint32_t seed_stride) {
    CHECK_ARG(e, "null env");
    HIP_TRY(hipSetDevice(e->ctx->device));
    int rc = sync_env(e);
    if (rc) return rc;
    const bool refill = enabled && e->ready && (!e->autoreset || e->stride != seed_stride);
    e->autoreset = enabled ? 1 : 0;
    e->stride = seed_stride;
    if (refill)  // the queued next episodes depend on the stride
        return with_shape(e->ctx->shape, [&](auto cf) { return fill_next_slots<decltype(cf)>(e); });
    return M3_OK;
}

int m3_env_step_device(m3_env* e, const int32_t* d_actions) {
    CHECK_ARG(e, "null env");
    if (!e->ready)
        return set_err(M3_ERR_STATE, "m3_env_step before m3_env_reset (or before m3_env_set of boards, seeds, "
                                     "score, moves and next_action)");
    HIP_TRY(hipSetDevice(e->ctx->device));
    return with_shape(e->ctx->shape, [&](auto cf) {
        if (e->stale) {
            const int rc = rederive<decltype(cf)>(e);
            if (rc) return rc;
        }
        return launch_env_step<decltype(cf)>(e, d_actions);
    });
}

// Host actions: copied into pinned staging[p] (p = step parity) on the host,
// uploaded to actions[p] on the upload stream, which waits only for the
// shards of step t-2 (the last readers of actions[p]) -- not for step t-1 and
// not for an RCCL gather on the context stream. The host blocks only until
// the upload of step t-2 has left staging[p].
int m3_env_step(m3_env* e, const int32_t* actions) {
    CHECK_ARG(e, "null env");
    if (!actions) return m3_env_step_device(e, nullptr);
    if (!e->ready)
        return set_err(M3_ERR_STATE, "m3_env_step before m3_env_reset (or before m3_env_set of boards, seeds, "
                                     "score, moves and next_action)");
    HIP_TRY(hipSetDevice(e->ctx->device));
    // a loaded env rederives (and restarts the step counter) before the upload buffer's parity is
    // chosen: the kernel of this step reads actions[steps & 1] of the counter it runs under
    int rc0 = ensure_fresh(e);
    if (rc0) return rc0;
    const size_t bytes = (size_t)e->n * 4;
    if (!e->ustream) {
        HIP_TRY(hipStreamCreateWithFlags(&e->ustream, hipStreamNonBlocking));
        for (int p = 0; p < 2; ++p) {
            HIP_TRY(hipEventCreateWithFlags(&e->upload_ev[p], hipEventDisableTiming));
            HIP_TRY(hipMalloc(&e->actions[p], bytes));
            HIP_TRY(hipHostMalloc(&e->hstage[p], bytes, hipHostMallocDefault));
        }
    }
    const int pb = (int)(e->steps & 1);
    if (e->upload_pend[pb]) {  // staging[pb] still feeding the upload of step t-2
        HIP_TRY(hipEventSynchronize(e->upload_ev[pb]));
        e->upload_pend[pb] = false;
    }
    memcpy(e->hstage[pb], actions, bytes);
    for (auto& sh : e->shards)
        if (sh.n && sh.apending[pb]) HIP_TRY(hipStreamWaitEvent(e->ustream, sh.aev[pb], 0));
    HIP_TRY(hipMemcpyAsync(e->actions[pb], e->hstage[pb], bytes, hipMemcpyHostToDevice, e->ustream));
    HIP_TRY(hipEventRecord(e->upload_ev[pb], e->ustream));
    e->upload_pend[pb] = true;
    e->upload_this = true;
    const int rc = m3_env_step_device(e, e->actions[pb]);
    e->upload_this = false;
    return rc;
}

static int env_field(m3_env* e, int what, void** ptr, size_t* bytes) {
    const int64_t n = e->n;
    switch (what) {
        case M3_ENV_BOARDS: *ptr = e->boards[e->cur]; *bytes = n * (size_t)e->ctx->N; return M3_OK;
        case M3_ENV_REWARD: *ptr = e->reward; *bytes = n * 4; return M3_OK;
        case M3_ENV_DONE: *ptr = e->done; *bytes = n; return M3_OK;
        case M3_ENV_TRUNCATED: *ptr = e->trunc; *bytes = n; return M3_OK;
        case M3_ENV_SCORE: *ptr = e->score; *bytes = n * 4; return M3_OK;
        case M3_ENV_MOVES: *ptr = e->moves; *bytes = n * 4; return M3_OK;
        case M3_ENV_FLAGS: *ptr = e->flags; *bytes = n * 4; return M3_OK;
        case M3_ENV_NEXT_ACTION: *ptr = e->next_action; *bytes = n * 4; return M3_OK;
        case M3_ENV_LEGAL: *ptr = e->legal; *bytes = n * 4ull * e->ctx->AW; return M3_OK;
        case M3_ENV_SEEDS: *ptr = e->seeds; *bytes = n * 4; return M3_OK;
        case M3_ENV_DRAWS: *ptr = e->draws; *bytes = n * 4; return M3_OK;
        case M3_ENV_GATHERED:
            if (!e->gathered) return set_err(M3_ERR_STATE, "M3_ENV_GATHERED before m3_env_comm_init");
            *ptr = e->gathered;
            *bytes = (size_t)e->nranks * n * 4;
            return M3_OK;
        default: return set_err(M3_ERR_INVALID, "unknown env field %d", what);
    }
}

int m3_env_get(m3_env* e, int what, void* host_out) {
    CHECK_ARG(e && host_out, "bad arguments");
    void* p;
    size_t bytes;
    int rc = env_field(e, what, &p, &bytes);
    if (rc) return rc;
    HIP_TRY(hipSetDevice(e->ctx->device));
    rc = ensure_fresh(e);
    if (rc) return rc;
    rc = join_shards(e, e->ctx->stream);
    if (rc) return rc;
    if (what == M3_ENV_LEGAL && !e->legal_eager) {  // derived on request from the current boards
        rc = with_shape(e->ctx->shape, [&](auto cf) {
            return launch_legal<decltype(cf)>(e->ctx, e->n, e->boards[e->cur], e->legal);
        });
        if (rc) return rc;
    }
    HIP_TRY(hipMemcpyAsync(host_out, p, bytes, hipMemcpyDeviceToHost, e->ctx->stream));
    HIP_TRY(hipStreamSynchronize(e->ctx->stream));
    return M3_OK;
}

int m3_env_set(m3_env* e, int what, const void* host_in) {
    CHECK_ARG(e && host_in, "bad arguments");
    switch (what) {
        case M3_ENV_BOARDS: case M3_ENV_SEEDS: case M3_ENV_SCORE: case M3_ENV_MOVES: case M3_ENV_NEXT_ACTION:
        case M3_ENV_REWARD: case M3_ENV_DONE: case M3_ENV_TRUNCATED: case M3_ENV_FLAGS: case M3_ENV_DRAWS:
            break;
        default:
            return set_err(M3_ERR_INVALID, "env field %d is derived, not settable", what);
    }
    void* p;
    size_t bytes;
    int rc = env_field(e, what, &p, &bytes);
    if (rc) return rc;
    if (what == M3_ENV_BOARDS) {
        const int8_t* b = static_cast<const int8_t*>(host_in);
        for (size_t i = 0; i < bytes; ++i)
            if (b[i] < 0) return set_err(M3_ERR_INVALID, "cell value outside [0, 127] at byte %zu", i);
    }
    HIP_TRY(hipSetDevice(e->ctx->device));
    rc = sync_env(e);
    if (rc) return rc;
    HIP_TRY(hipMemcpy(p, host_in, bytes, hipMemcpyHostToDevice));
    e->stale = true;
    // stepping needs the whole state: after a reset any field may be overwritten; a fresh env is
    // ready once boards, seeds, score, moves and the pre-drawn action have all been loaded
    constexpr uint32_t NEED = (1u << M3_ENV_BOARDS) | (1u << M3_ENV_SEEDS) | (1u << M3_ENV_SCORE) |
                              (1u << M3_ENV_MOVES) | (1u << M3_ENV_NEXT_ACTION);
    e->loaded |= 1u << what;
    if ((e->loaded & NEED) == NEED) e->ready = true;
    return M3_OK;
}

int m3_env_comm_size(m3_env* e, int* out) {
    CHECK_ARG(e && out, "bad arguments");
    if (!e->comm) {
        *out = 1;
        return M3_OK;
    }
    int n = 0;
    RCCL_TRY(ncclCommCount(e->comm, &n));
    *out = n;
    return M3_OK;
}

int m3_env_device_ptr(m3_env* e, int what, void** out) {
    CHECK_ARG(e && out, "bad arguments");
    size_t bytes;
    int rc = env_field(e, what, out, &bytes);
    if (rc || what != M3_ENV_LEGAL || e->legal_eager) return rc;
    // a device consumer of the legal sets: from now on every step writes them; fill the buffer now
    HIP_TRY(hipSetDevice(e->ctx->device));
    rc = ensure_fresh(e);
    if (rc) return rc;
    rc = join_shards(e, e->ctx->stream);
    if (rc) return rc;
    rc = with_shape(e->ctx->shape, [&](auto cf) {
        return launch_legal<decltype(cf)>(e->ctx, e->n, e->boards[e->cur], e->legal);
    });
    if (rc) return rc;
    HIP_TRY(hipStreamSynchronize(e->ctx->stream));
    e->legal_eager = true;
    return M3_OK;
}

int m3_comm_unique_id(uint8_t out_id[128]) {
    CHECK_ARG(out_id, "null out");
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
    ncclUniqueId id;
    RCCL_TRY(ncclGetUniqueId(&id));
    memcpy(out_id, &id, 128);
    return M3_OK;
}

int m3_env_comm_init(m3_env* e, const uint8_t id[128], int nranks, int rank) {
    CHECK_ARG(e && id && nranks >= 1 && rank >= 0 && rank < nranks, "bad arguments");
    if (e->comm) return set_err(M3_ERR_STATE, "m3_env_comm_init: the env already has a communicator");
    HIP_TRY(hipSetDevice(e->ctx->device));
    int32_t* g = nullptr;
    HIP_TRY(hipMalloc(&g, (size_t)nranks * e->n * 4));
    ncclUniqueId uid;
    memcpy(&uid, id, 128);
    ncclComm_t comm = nullptr;
    const ncclResult_t r = ncclCommInitRank(&comm, nranks, uid, rank);
    if (r != ncclSuccess) {
        (void)hipFree(g);
        return set_err(M3_ERR_RCCL, "ncclCommInitRank: %s", ncclGetErrorString(r));
    }
    e->comm = comm;
    e->gathered = g;
    e->nranks = nranks;
    e->rank = rank;
    return M3_OK;
}

// ncclAllGather of the last step's packed words on the context stream into
// d_out (nullptr: the env's own buffer, M3_ENV_GATHERED).
static int env_gather(m3_env* e, int32_t* d_out) {
    if (!e->comm) return set_err(M3_ERR_STATE, "m3_env_gather before m3_env_comm_init");
    if (e->steps == 0) return set_err(M3_ERR_STATE, "m3_env_gather before the first m3_env_step");
    HIP_TRY(hipSetDevice(e->ctx->device));
    int rc = join_shards(e, e->ctx->stream);  // every shard's packed words written
    if (rc) return rc;
    const int pb = (int)((e->steps - 1) & 1);  // buffer the last step wrote
    RCCL_TRY(ncclAllGather(e->packed + (size_t)pb * e->n, d_out ? d_out : e->gathered, (size_t)e->n, ncclInt32,
                           e->comm, e->ctx->stream));
    HIP_TRY(hipEventRecord(e->gev[pb], e->ctx->stream));  // the step after next must not overwrite it early
    e->gpend[pb] = true;
    return M3_OK;
}

int m3_env_gather(m3_env* e, int32_t* host_out) {
    CHECK_ARG(e, "null env");
    int rc = env_gather(e, nullptr);
    if (rc) return rc;
    if (host_out) {
        HIP_TRY(hipMemcpyAsync(host_out, e->gathered, (size_t)e->nranks * e->n * 4, hipMemcpyDeviceToHost,
                               e->ctx->stream));
        HIP_TRY(hipStreamSynchronize(e->ctx->stream));
    }
    return M3_OK;
}

int m3_env_gather_device(m3_env* e, int32_t* d_out) {
    CHECK_ARG(e, "null env");
    return env_gather(e, d_out);
}

}  // extern "C"

// Test hook kernel: one wave sleeping ~`rounds` x 8k cycles.
__global__ void k_stall(uint32_t rounds) {
    for (uint32_t i = 0; i < rounds; ++i) __builtin_amdgcn_s_sleep(127);
}

extern "C" {

int m3_env_debug_stall(m3_env* e, uint32_t usec) {
    CHECK_ARG(e && usec <= 10u * 1000u * 1000u, "bad arguments");
    HIP_TRY(hipSetDevice(e->ctx->device));
    // s_sleep 127 = 127 x 64 clocks, ~3.4 us at 2.4 GHz
    hipLaunchKernelGGL(k_stall, dim3(1), dim3(64), 0, e->ctx->stream, (usec + 2u) / 3u);
    HIP_TRY(hipGetLastError());
    return M3_OK;
}

int m3_env_stats(m3_env* e, uint64_t out[4]) {
    CHECK_ARG(e && out, "bad arguments");
    HIP_TRY(hipSetDevice(e->ctx->device));
    int rc = sync_env(e);
    if (rc) return rc;
    std::vector<uint32_t> h(64 * MAX_SHARDS);
    HIP_TRY(hipMemcpy(h.data(), e->counters, h.size() * 4, hipMemcpyDeviceToHost));
    out[0] = out[1] = out[2] = out[3] = 0;
    for (size_t s = 0; s < e->shards.size(); ++s) {
        out[0] += h[64 * s + 40];  // steps recomputed (cache exhausted or > table groups)
        out[1] += h[64 * s + 42];  // resets recomputed by the wave-cooperative pass (>= 624 draws)
        out[2] += h[64 * s + 41];  // autoresets (episodes prefetched)
    }
    out[3] = e->shards.size();
    return M3_OK;
}

#ifdef M3_PHASE_PROF
// profiling build only (not part of include/m3.h): out[2][PH_N + 2], summed over the
// configurations' translation units (each has its own g_prof)
#ifdef M3_SPLIT_TU
#ifdef M3_HEADLINE_ONLY
extern "C" int m3_prof_read_0(uint64_t*, int), m3_prof_read_1(uint64_t*, int);
int m3_prof_read(uint64_t* out, int reset) {
    int (*const rd[2])(uint64_t*, int) = {m3_prof_read_0, m3_prof_read_1};
#else
extern "C" int m3_prof_read_0(uint64_t*, int), m3_prof_read_1(uint64_t*, int), m3_prof_read_2(uint64_t*, int),
    m3_prof_read_3(uint64_t*, int), m3_prof_read_4(uint64_t*, int), m3_prof_read_5(uint64_t*, int),
    m3_prof_read_6(uint64_t*, int), m3_prof_read_7(uint64_t*, int), m3_prof_read_8(uint64_t*, int),
    m3_prof_read_9(uint64_t*, int);
int m3_prof_read(uint64_t* out, int reset) {
    static_assert(N_CONFIGS == 10, "one reader per configuration");
    int (*const rd[10])(uint64_t*, int) = {m3_prof_read_0, m3_prof_read_1, m3_prof_read_2, m3_prof_read_3,
                                          m3_prof_read_4, m3_prof_read_5, m3_prof_read_6, m3_prof_read_7,
                                          m3_prof_read_8, m3_prof_read_9};
#endif
    uint64_t part[2 * PROF_SLOTS];
    for (int i = 0; i < 2 * PROF_SLOTS; ++i) out[i] = 0;
    for (auto f : rd) {
        const int rc = f(part, reset);
        if (rc < 0) return rc;
        for (int i = 0; i < 2 * PROF_SLOTS; ++i) out[i] += part[i];
    }
    return PH_N;
}
#else
int m3_prof_read(uint64_t* out, int reset) { return m3_prof_read_tu(out, reset); }
#endif
#endif

int m3_env_timing(m3_env* e, int capacity) {
    CHECK_ARG(e && capacity >= 0, "bad arguments");
    HIP_TRY(hipSetDevice(e->ctx->device));
    int rc = sync_env(e);
    if (rc) return rc;
    while ((int)e->tev.size() < 3 * capacity) {
        hipEvent_t ev;
        HIP_TRY(hipEventCreate(&ev));
        e->tev.push_back(ev);
    }
    e->tcap = capacity;
    e->tn = 0;
    return M3_OK;
}

int m3_env_kernel_ms(m3_env* e, float* out_ms, int max_n, int* out_n) {
    CHECK_ARG(e && out_n && (max_n == 0 || out_ms), "bad arguments");
    HIP_TRY(hipSetDevice(e->ctx->device));
    const int n = e->tn < max_n ? e->tn : max_n;
    int rc = sync_env(e);
    if (rc) return rc;
    for (int i = 0; i < n; ++i) HIP_TRY(hipEventElapsedTime(&out_ms[i], e->tev[3 * i], e->tev[3 * i + 2]));
    *out_n = n;
    return M3_OK;
}

int m3_env_step_kernel_ms(m3_env* e, float* out_ms, int max_n, int* out_n) {
    CHECK_ARG(e && out_n && (max_n == 0 || out_ms), "bad arguments");
    HIP_TRY(hipSetDevice(e->ctx->device));
    const int n = e->tn < max_n ? e->tn : max_n;
    int rc = sync_env(e);
    if (rc) return rc;
    for (int i = 0; i < n; ++i) HIP_TRY(hipEventElapsedTime(&out_ms[i], e->tev[3 * i], e->tev[3 * i + 1]));
    *out_n = n;
    return M3_OK;
}

}  // extern "C"
