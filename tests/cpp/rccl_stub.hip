// rccl_stub.hip — TEST-ONLY stand-in for the RCCL entry points that
// libgsplat's one-process group (csrc/host/group.cpp, GS_TRANSPORT_RCCL)
// resolves with dlopen.  It is loaded only when GS_RCCL_LIB names it
// (tests/test_gpu_group.py::test_group_rccl_stub_*), so the RCCL branch of
// every group collective runs on a one-GPU box: ranks may share a device, and
// each collective becomes stream-ordered peer copies (plus, for the sums, a
// small kernel adding the ranks' buffers in rank order, the order of the copy
// transport's accumulate).  Never shipped, never a fallback: the product
// loads the real librccl unless a test points GS_RCCL_LIB here.
//
// Semantics kept from RCCL: calls inside ncclGroupStart/End are collected
// and issued at the outermost ncclGroupEnd; a send matches the recv of the
// same (sender, receiver) pair in issue order, with equal byte counts; a
// collective needs one call per rank of the communicator set.  Each transfer
// waits for the work queued before it on the source's stream and holds back
// later work on both streams until it is done.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <vector>

namespace {

struct World;
}  // namespace

struct ncclComm {
    int rank = 0, nranks = 0, dev = 0;
    World* world = nullptr;
};

namespace {

struct Op {
    enum Kind { SEND, RECV, ALLREDUCE, ALLGATHER, REDUCE } kind;
    const void* sbuf;
    void* rbuf;
    size_t bytes;  // per rank (send / recv / all-gather chunk / reduce vector)
    ncclDataType_t dt;
    int peer;  // send: receiver, recv: sender, reduce: root
    ncclComm* comm;
    hipStream_t st;
};

struct World {
    int n = 0;
    std::vector<ncclComm*> comms;
    int refs = 0;
};

int g_depth = 0;
std::vector<Op> g_ops;

size_t type_size(ncclDataType_t t) {
    switch (t) {
    case ncclInt8: case ncclUint8: return 1;
    case ncclFloat16: case ncclBfloat16: return 2;
    case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
    case ncclInt64: case ncclUint64: case ncclFloat64: return 8;
    default: return 0;
    }
}

template <typename T>
__global__ void add_kernel(T* __restrict__ dst, const T* __restrict__ src, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = dst[i] + src[i];
}

hipError_t launch_add(void* dst, const void* src, size_t bytes, ncclDataType_t t, hipStream_t st) {
    const size_t es = type_size(t), n = bytes / es;
    const unsigned grid = (unsigned)std::min<size_t>((n + 255) / 256, 4096);
    if (!n) return hipSuccess;
    switch (t) {
    case ncclFloat32: add_kernel<float><<<grid, 256, 0, st>>>((float*)dst, (const float*)src, n); break;
    case ncclFloat64: add_kernel<double><<<grid, 256, 0, st>>>((double*)dst, (const double*)src, n); break;
    case ncclUint64: add_kernel<unsigned long long><<<grid, 256, 0, st>>>((unsigned long long*)dst, (const unsigned long long*)src, n); break;
    case ncclInt64: add_kernel<long long><<<grid, 256, 0, st>>>((long long*)dst, (const long long*)src, n); break;
    case ncclUint32: add_kernel<unsigned><<<grid, 256, 0, st>>>((unsigned*)dst, (const unsigned*)src, n); break;
    case ncclInt32: add_kernel<int><<<grid, 256, 0, st>>>((int*)dst, (const int*)src, n); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

#define STUB_HIP(x)                                   \
    do {                                              \
        if ((x) != hipSuccess) return ncclUnhandledCudaError; \
    } while (0)

// b's stream waits for the work queued on a's stream so far (a may be b).
ncclResult_t order(hipStream_t a, int adev, hipStream_t b, int bdev) {
    if (a == b) return ncclSuccess;
    hipEvent_t e;
    STUB_HIP(hipSetDevice(adev));
    STUB_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    STUB_HIP(hipEventRecord(e, a));
    STUB_HIP(hipSetDevice(bdev));
    STUB_HIP(hipStreamWaitEvent(b, e, 0));
    STUB_HIP(hipEventDestroy(e));  // (released once the wait is satisfied)
    return ncclSuccess;
}

ncclResult_t copy(void* dst, int ddev, const void* src, int sdev, size_t bytes, hipStream_t st) {
    if (!bytes) return ncclSuccess;
    STUB_HIP(hipSetDevice(ddev));
    STUB_HIP(hipMemcpyPeerAsync(dst, ddev, src, sdev, bytes, st));
    return ncclSuccess;
}

#define STUB_OK(x)                                  \
    do {                                            \
        ncclResult_t r_ = (x);                      \
        if (r_ != ncclSuccess) return r_;           \
    } while (0)

// One collective: the ops of kind k from every rank of the world, by rank.
ncclResult_t run_collective(std::vector<const Op*>& by_rank) {
    const int n = (int)by_rank.size();
    const Op& o0 = *by_rank[0];
    for (const Op* o : by_rank)
        if (!o || o->bytes != o0.bytes || o->dt != o0.dt || (o0.kind == Op::REDUCE && o->peer != o0.peer))
            return ncclInvalidUsage;
    if (o0.kind == Op::ALLGATHER) {
        // rank d's recv buffer = [rank 0's chunk, ..., rank n-1's chunk]
        for (int d = 0; d < n; ++d) {
            const Op& od = *by_rank[(size_t)d];
            for (int j = 0; j < n; ++j) {
                const Op& oj = *by_rank[(size_t)j];
                STUB_OK(order(oj.st, oj.comm->dev, od.st, od.comm->dev));
                STUB_OK(copy((char*)od.rbuf + (size_t)j * o0.bytes, od.comm->dev, oj.sbuf, oj.comm->dev, o0.bytes, od.st));
            }
        }
        for (int j = 0; j < n; ++j)  // (a rank's send buffer is free once every copy of it is done)
            for (int d = 0; d < n; ++d)
                STUB_OK(order(by_rank[(size_t)d]->st, by_rank[(size_t)d]->comm->dev, by_rank[(size_t)j]->st,
                              by_rank[(size_t)j]->comm->dev));
        return ncclSuccess;
    }
    // sums: accumulated on the root's (reduce) or rank 0's device and stream,
    // acc = buf 0, acc += buf 1, ... (rank order)
    const int root = o0.kind == Op::REDUCE ? o0.peer : 0;
    if (root < 0 || root >= n) return ncclInvalidArgument;
    const Op& orr = *by_rank[(size_t)root];
    const int rdev = orr.comm->dev;
    hipStream_t rst = orr.st;
    void *acc = nullptr, *tmp = nullptr;
    STUB_HIP(hipSetDevice(rdev));
    STUB_HIP(hipMalloc(&acc, o0.bytes ? o0.bytes : 1));
    STUB_HIP(hipMalloc(&tmp, o0.bytes ? o0.bytes : 1));
    for (int j = 0; j < n; ++j) {
        const Op& oj = *by_rank[(size_t)j];
        STUB_OK(order(oj.st, oj.comm->dev, rst, rdev));
        STUB_OK(copy(j == 0 ? acc : tmp, rdev, oj.sbuf, oj.comm->dev, o0.bytes, rst));
        if (j > 0) {
            STUB_HIP(hipSetDevice(rdev));
            STUB_HIP(launch_add(acc, tmp, o0.bytes, o0.dt, rst));
        }
    }
    if (o0.kind == Op::REDUCE) {
        STUB_OK(copy(orr.rbuf, rdev, acc, rdev, o0.bytes, rst));
    } else {
        for (int d = 0; d < n; ++d) STUB_OK(copy(by_rank[(size_t)d]->rbuf, by_rank[(size_t)d]->comm->dev, acc, rdev, o0.bytes, rst));
    }
    for (int j = 0; j < n; ++j) STUB_OK(order(rst, rdev, by_rank[(size_t)j]->st, by_rank[(size_t)j]->comm->dev));
    STUB_HIP(hipSetDevice(rdev));
    STUB_HIP(hipStreamSynchronize(rst));  // (test stub: the scratch goes at once)
    STUB_HIP(hipFree(acc));
    STUB_HIP(hipFree(tmp));
    return ncclSuccess;
}

ncclResult_t flush() {
    std::vector<Op> ops;
    ops.swap(g_ops);
    // point-to-point: each recv takes the first unmatched send of its pair
    std::vector<bool> used(ops.size(), false);
    for (size_t i = 0; i < ops.size(); ++i) {
        const Op& r = ops[i];
        if (r.kind != Op::RECV) continue;
        size_t j = 0;
        for (; j < ops.size(); ++j)
            if (!used[j] && ops[j].kind == Op::SEND && ops[j].comm->world == r.comm->world &&
                ops[j].comm->rank == r.peer && ops[j].peer == r.comm->rank)
                break;
        if (j == ops.size()) return ncclInvalidUsage;
        const Op& s = ops[j];
        if (s.bytes != r.bytes) return ncclInvalidArgument;
        used[i] = used[j] = true;
        STUB_OK(order(s.st, s.comm->dev, r.st, r.comm->dev));
        STUB_OK(copy(r.rbuf, r.comm->dev, s.sbuf, s.comm->dev, r.bytes, r.st));
        STUB_OK(order(r.st, r.comm->dev, s.st, s.comm->dev));
    }
    for (size_t i = 0; i < ops.size(); ++i)
        if (ops[i].kind == Op::SEND && !used[i]) return ncclInvalidUsage;
    // collectives: the k-th collective call of each rank forms the k-th collective
    for (Op::Kind k : {Op::ALLREDUCE, Op::ALLGATHER, Op::REDUCE}) {
        std::vector<std::vector<const Op*>> per;  // per[c][rank]
        std::vector<int> next;
        for (const Op& o : ops) {
            if (o.kind != k) continue;
            const int n = o.comm->nranks, rk = o.comm->rank;
            if (next.empty()) next.assign((size_t)n, 0);
            const int c = next[(size_t)rk]++;
            if ((int)per.size() <= c) per.resize((size_t)c + 1, std::vector<const Op*>((size_t)n, nullptr));
            per[(size_t)c][(size_t)rk] = &o;
        }
        for (auto& by_rank : per) STUB_OK(run_collective(by_rank));
    }
    return ncclSuccess;
}

ncclResult_t push(const Op& o) {
    if (!o.comm || !o.comm->world) return ncclInvalidArgument;
    g_ops.push_back(o);
    return g_depth > 0 ? ncclSuccess : flush();
}

}  // namespace

extern "C" {

// The group may place ranks on one device with this library (test stub).
int gs_rccl_stub_shared_devices() { return 1; }

ncclResult_t ncclCommInitAll(ncclComm_t* comm, int ndev, const int* devlist) {
    if (!comm || ndev <= 0) return ncclInvalidArgument;
    World* w = new World;
    w->n = ndev;
    w->refs = ndev;
    for (int i = 0; i < ndev; ++i) {
        ncclComm* c = new ncclComm;
        c->rank = i;
        c->nranks = ndev;
        c->dev = devlist ? devlist[i] : i;
        c->world = w;
        w->comms.push_back(c);
        comm[i] = c;
    }
    return ncclSuccess;
}

static ncclResult_t release(ncclComm_t c) {
    if (!c) return ncclInvalidArgument;
    World* w = c->world;
    delete c;
    if (w && --w->refs == 0) delete w;
    return ncclSuccess;
}
ncclResult_t ncclCommDestroy(ncclComm_t comm) { return release(comm); }
ncclResult_t ncclCommAbort(ncclComm_t comm) { return release(comm); }

ncclResult_t ncclCommGetAsyncError(ncclComm_t comm, ncclResult_t* asyncError) {
    if (!comm || !asyncError) return ncclInvalidArgument;
    *asyncError = ncclSuccess;
    return ncclSuccess;
}

const char* ncclGetErrorString(ncclResult_t r) {
    switch (r) {
    case ncclSuccess: return "no error (rccl stub)";
    case ncclUnhandledCudaError: return "HIP call failed (rccl stub)";
    case ncclInvalidArgument: return "invalid argument (rccl stub)";
    case ncclInvalidUsage: return "invalid usage: unmatched send/recv or collective (rccl stub)";
    default: return "error (rccl stub)";
    }
}

ncclResult_t ncclGroupStart() {
    ++g_depth;
    return ncclSuccess;
}
ncclResult_t ncclGroupEnd() {
    if (g_depth <= 0) return ncclInvalidUsage;
    return --g_depth == 0 ? flush() : ncclSuccess;
}

ncclResult_t ncclSend(const void* sendbuff, size_t count, ncclDataType_t datatype, int peer, ncclComm_t comm,
                      hipStream_t stream) {
    return push(Op{Op::SEND, sendbuff, nullptr, count * type_size(datatype), datatype, peer, comm, stream});
}
ncclResult_t ncclRecv(void* recvbuff, size_t count, ncclDataType_t datatype, int peer, ncclComm_t comm,
                      hipStream_t stream) {
    return push(Op{Op::RECV, nullptr, recvbuff, count * type_size(datatype), datatype, peer, comm, stream});
}
ncclResult_t ncclAllReduce(const void* sendbuff, void* recvbuff, size_t count, ncclDataType_t datatype, ncclRedOp_t op,
                           ncclComm_t comm, hipStream_t stream) {
    if (op != ncclSum) return ncclInvalidArgument;
    return push(Op{Op::ALLREDUCE, sendbuff, recvbuff, count * type_size(datatype), datatype, 0, comm, stream});
}
ncclResult_t ncclAllGather(const void* sendbuff, void* recvbuff, size_t sendcount, ncclDataType_t datatype,
                           ncclComm_t comm, hipStream_t stream) {
    return push(Op{Op::ALLGATHER, sendbuff, recvbuff, sendcount * type_size(datatype), datatype, 0, comm, stream});
}
ncclResult_t ncclReduce(const void* sendbuff, void* recvbuff, size_t count, ncclDataType_t datatype, ncclRedOp_t op,
                        int root, ncclComm_t comm, hipStream_t stream) {
    if (op != ncclSum) return ncclInvalidArgument;
    return push(Op{Op::REDUCE, sendbuff, recvbuff, count * type_size(datatype), datatype, root, comm, stream});
}

}  // extern "C"
