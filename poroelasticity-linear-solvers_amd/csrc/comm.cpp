// comm.cpp -- CommSelf / CommCallback / CommRCCL (see comm.hpp).
#include "comm.hpp"

#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <string>

#include "runtime.hpp"

namespace pls {

#define NCCLCHK(x)                                                                                  \
    do {                                                                                            \
        ncclResult_t r_ = (x);                                                                      \
        if (r_ != ncclSuccess)                                                                      \
            throw ::pls::Error(std::string(#x) + " failed: " + ncclGetErrorString(r_));             \
    } while (0)

// rank-ordered sum of the gathered partials: out[j] = sum_r g[r * count + j]
__global__ void k_ordered_sum(int size, int count, const double *g, double *out) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= count) return;
    double s = 0.0;
    for (int r = 0; r < size; ++r) s += g[(int64_t)r * count + j];
    out[j] = s;
}

void Comm::global_sum_dev(double *d_vals, int count, hipStream_t st) {
    if (size == 1 || count <= 0) return;
    const size_t need = (size_t)size * count;
    if (need > scratch_n_) {
        if (scratch_) (void)hipFree(scratch_);
        HIPCHK(hipMalloc((void **)&scratch_, sizeof(double) * need));
        scratch_n_ = need;
    }
    allgather_dev(d_vals, count, scratch_, st);
    k_ordered_sum<<<(count + 255) / 256, 256, 0, st>>>(size, count, scratch_, d_vals);
    HIPCHK(hipGetLastError());
}

void Comm::alltoallv_i64(const std::vector<std::vector<int64_t>> &to, std::vector<std::vector<int64_t>> &from) {
    // message of rank r: [count to each peer][payloads in peer order]; padded allgather
    std::vector<int64_t> msg(size, 0);
    for (int p = 0; p < size; ++p) msg[p] = (int64_t)to[p].size();
    for (int p = 0; p < size; ++p) msg.insert(msg.end(), to[p].begin(), to[p].end());
    int64_t len = (int64_t)msg.size();
    std::vector<int64_t> lens(size);
    allgather_host(&len, sizeof(int64_t), lens.data());
    const int64_t mx = *std::max_element(lens.begin(), lens.end());
    msg.resize(mx, 0);
    std::vector<int64_t> all((size_t)mx * size);
    allgather_host(msg.data(), mx * (int64_t)sizeof(int64_t), all.data());
    from.assign(size, {});
    for (int p = 0; p < size; ++p) {
        const int64_t *m = all.data() + (size_t)p * mx;
        int64_t off = size;
        for (int q = 0; q < rank; ++q) off += m[q];
        from[p].assign(m + off, m + off + m[rank]);
    }
}

// ------------------------------------------------------------------ self --
void CommSelf::allgather_dev(const double *d_send, int count, double *d_recv, hipStream_t st) {
    if (d_recv != d_send) HIPCHK(hipMemcpyAsync(d_recv, d_send, sizeof(double) * count, hipMemcpyDeviceToDevice, st));
}
void CommSelf::allgather_host(const void *send, int64_t bytes, void *recv) { std::memcpy(recv, send, bytes); }

// -------------------------------------------------------------- callback --
void CommCallback::allgather_host(const void *send, int64_t bytes, void *recv) {
    if (fn(send, bytes, recv, user) != 0) throw Error("communicator callback (allgather) failed");
}
void CommCallback::allgather_dev(const double *d_send, int count, double *d_recv, hipStream_t st) {
    std::vector<double> h(count), all((size_t)count * size);
    HIPCHK(hipMemcpyAsync(h.data(), d_send, sizeof(double) * count, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    allgather_host(h.data(), sizeof(double) * count, all.data());
    HIPCHK(hipMemcpyAsync(d_recv, all.data(), sizeof(double) * all.size(), hipMemcpyHostToDevice, st));
    HIPCHK(hipStreamSynchronize(st));
}
void CommCallback::exchange_dev(const double *d_send, const std::vector<int64_t> &scnt,
                                const std::vector<int64_t> &soff, double *d_recv, const std::vector<int64_t> &rcnt,
                                const std::vector<int64_t> &roff, hipStream_t st) {
    int64_t ns = 0;
    for (int p = 0; p < size; ++p) ns = std::max(ns, soff[p] + scnt[p]);
    std::vector<double> hs(ns);
    if (ns) HIPCHK(hipMemcpyAsync(hs.data(), d_send, sizeof(double) * ns, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    // message: [scnt per peer][segments in peer order]
    std::vector<double> msg(size);
    for (int p = 0; p < size; ++p) msg[p] = (double)scnt[p];
    for (int p = 0; p < size; ++p) msg.insert(msg.end(), hs.begin() + soff[p], hs.begin() + soff[p] + scnt[p]);
    int64_t len = (int64_t)msg.size();
    std::vector<int64_t> lens(size);
    allgather_host(&len, sizeof(int64_t), lens.data());
    const int64_t mx = *std::max_element(lens.begin(), lens.end());
    msg.resize(mx, 0.0);
    std::vector<double> all((size_t)mx * size);
    allgather_host(msg.data(), mx * (int64_t)sizeof(double), all.data());
    int64_t nr = 0;
    for (int p = 0; p < size; ++p) nr = std::max(nr, roff[p] + rcnt[p]);
    std::vector<double> hr(nr, 0.0);
    for (int p = 0; p < size; ++p) {
        if (p == rank || rcnt[p] == 0) continue;
        const double *m = all.data() + (size_t)p * mx;
        int64_t off = size;
        for (int q = 0; q < rank; ++q) off += (int64_t)m[q];
        if ((int64_t)m[rank] != rcnt[p]) throw Error("halo exchange: count mismatch");
        std::copy(m + off, m + off + rcnt[p], hr.begin() + roff[p]);
    }
    if (nr) HIPCHK(hipMemcpyAsync(d_recv, hr.data(), sizeof(double) * nr, hipMemcpyHostToDevice, st));
    HIPCHK(hipStreamSynchronize(st));
}

// ------------------------------------------------------------------ RCCL --
CommRCCL::~CommRCCL() {
    if (nccl) (void)ncclCommDestroy((ncclComm_t)nccl);
}
void CommRCCL::allgather_dev(const double *d_send, int count, double *d_recv, hipStream_t st) {
    NCCLCHK(ncclAllGather(d_send, d_recv, (size_t)count, ncclDouble, (ncclComm_t)nccl, st));
}
void CommRCCL::exchange_dev(const double *d_send, const std::vector<int64_t> &scnt, const std::vector<int64_t> &soff,
                            double *d_recv, const std::vector<int64_t> &rcnt, const std::vector<int64_t> &roff,
                            hipStream_t st) {
    NCCLCHK(ncclGroupStart());
    for (int p = 0; p < size; ++p) {
        if (p == rank) continue;
        if (scnt[p]) NCCLCHK(ncclSend(d_send + soff[p], (size_t)scnt[p], ncclDouble, p, (ncclComm_t)nccl, st));
        if (rcnt[p]) NCCLCHK(ncclRecv(d_recv + roff[p], (size_t)rcnt[p], ncclDouble, p, (ncclComm_t)nccl, st));
    }
    NCCLCHK(ncclGroupEnd());
}
void CommRCCL::allgather_host(const void *send, int64_t bytes, void *recv) {
    char *d = nullptr;
    hipStream_t st;
    HIPCHK(hipStreamCreate(&st));
    HIPCHK(hipMalloc((void **)&d, (size_t)bytes * (size + 1)));
    HIPCHK(hipMemcpy(d, send, bytes, hipMemcpyHostToDevice));
    NCCLCHK(ncclAllGather(d, d + bytes, (size_t)bytes, ncclChar, (ncclComm_t)nccl, st));
    HIPCHK(hipStreamSynchronize(st));
    HIPCHK(hipMemcpy(recv, d + bytes, (size_t)bytes * size, hipMemcpyDeviceToHost));
    (void)hipFree(d);
    (void)hipStreamDestroy(st);
}

int rccl_unique_id(char out[128]) {
    ncclUniqueId id;
    NCCLCHK(ncclGetUniqueId(&id));
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
    std::memcpy(out, &id, 128);
    return 0;
}

CommRCCL *rccl_init(const char idb[128], int rank, int size) {
    ncclUniqueId id;
    std::memcpy(&id, idb, 128);
    auto *c = new CommRCCL();
    c->rank = rank;
    c->size = size;
    ncclComm_t nc;
    NCCLCHK(ncclCommInitRank(&nc, size, id, rank));
    c->nccl = nc;
    return c;
}

}  // namespace pls
