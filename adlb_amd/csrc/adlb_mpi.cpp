// adlb_mpi.cpp -- libadlb.so: the ADLB application API (include/adlb/adlb.h)
// and the MPI server loop around the GPU work-queue engine.
//
// App side: the client halves of the reference's calls (src/adlb.c:2638-3068)
// with the same wire messages (adlb_wire.h), so every return code and the
// Put / Reserve / Get round trips behave as in the reference.
//
// Server side: one process per server rank runs ADLB_Server.  Each inbound
// message goes to the handler in adlb_core.cpp; runs of consecutive Reserves
// or Gets already waiting in MPI are drained into one GPU batch.  The
// reference's ring-passed control (qmstat table, no-more-work, end, exhaustion
// check; adlb.c:754-822, 1385-1650, 1705-1757) becomes direct messages between
// servers: each server sends its qmstat row to every other server every
// qmstat interval, and the master decides exhaustion from two consecutive
// all-idle polls with no queue activity in between.
//
// Steal group (the north star's cross-shard merge): when every
// server shares one node (or ADLB_STEAL_GROUP=1), parked Reserves are not
// stolen by SS_RFR / SS_RFR_RESP round trips (adlb.c:1280-1308, 1802-2050).
// Every ADLB_STEAL_INTERVAL s the master opens a round (SRV_STEAL to every
// server); each server exports its k best available units per type and its
// parked Reserves, the blobs are all-gathered among the servers
// (MPI_Allgather), and every server runs the same deterministic merge and
// settles its own side: answers its parked Reserves the round served, pins
// the units it donates.  A server takes no other message between its export
// and its settle, so the merge sees every queue as it is applied.
// ADLB_STEAL_GROUP=0 keeps the reference's SS_RFR protocol.
// Steal transport: when every server of the group owns a distinct GPU (PCI
// bus ids all-gathered at startup), the blobs stay in device memory and are
// all-gathered by RCCL over xGMI (the ncclUniqueId goes out by MPI_Bcast among
// the servers); otherwise, or if any server cannot load librccl (dlopen, so a
// relinked application needs RCCL only where it is used) or join the
// communicator, every server keeps the host MPI_Allgather.
// ADLB_STEAL_RCCL=0 forces MPI_Allgather, =1 tries RCCL even on a shared GPU.
// ADLB_STEAL_REPORT prints the transport chosen.
#include <mpi.h>

#include <dlfcn.h>
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>  // types only: the entry points come from dlopen (rccl_load)

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <unistd.h>
#include <vector>

#include "adlb/adlb.h"
#include "adlbq.h"
#include "adlb_core.h"
#include "adlb_wire.h"

namespace {

MPI_Comm g_all = MPI_COMM_NULL;  // dup of MPI_COMM_WORLD (adlb.c:317)
MPI_Comm g_srvcomm = MPI_COMM_NULL;  // the server ranks (steal-group all-gather)
int g_world = 0, g_rank = 0, g_S = 1, g_A = 0, g_master = 0, g_debug = -1;
int g_home = -1;  // an app's server (adlb.c:258)
int g_next_put = -1;
int g_dbgprintf = 0;
double g_t0 = 0.0;
std::vector<int> g_types;
// Begin/End_batch_put state of an app (adlb.c:2638-2752)
int g_common_len = 0, g_common_server = -1, g_common_seqno = -1, g_common_refcnt = 0, g_in_batch = 0;
adlbsrv *g_srv = nullptr;
bool g_is_server = false, g_is_debug = false;

int type_ok(int t) { return std::find(g_types.begin(), g_types.end(), t) != g_types.end(); }

double env_d(const char *name, double dflt) {
    const char *v = getenv(name);
    return v && *v ? atof(v) : dflt;
}

void die(const char *what) {
    fprintf(stderr, "%06d: ** ADLB server: %s\n", g_rank, what);
    fflush(stderr);
    MPI_Abort(MPI_COMM_WORLD, -1);
}

int next_put_server() {
    const int s = g_next_put++;
    if (g_next_put >= g_master + g_S) g_next_put = g_master;
    return s;
}

// ------------------------------------------------------------------ server loop
struct Pending {
    MPI_Request req;
    std::vector<char> buf;
};

struct Loop {
    std::vector<Pending *> pend;
    int my_idx = 0, my_apps = 0, apps_done = 0, servers_done = 0;
    bool done = false;
    // the qmstat table (rows of every server) as last received
    std::vector<int> qlen, hi;
    std::vector<double> nbytes;
    long long row_activity = -1;
    // exhaustion poll (master)
    int exh_epoch = 0, exh_wait = 0;
    bool exh_all_idle = true, exh_prev_idle = false;
    long long exh_sum = 0, exh_prev_sum = -1;
    // steal group
    bool group = false;
    bool steal_want = false;  // master: some server asked for a round (TAG_SRV_STEAL_WANT)
    std::vector<int> blob, blobs;
};
Loop *g_loop = nullptr;

// the steal round's device all-gather (RCCL)
struct Rccl {
    ncclComm_t comm = nullptr;
    int *d_blob = nullptr, *d_all = nullptr;
    hipStream_t st = nullptr;
} g_rccl;

// librccl's entry points, loaded on first use
struct RcclApi {
    void *lib = nullptr;
    ncclResult_t (*get_unique_id)(ncclUniqueId *) = nullptr;
    ncclResult_t (*comm_init_rank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*all_gather)(const void *, void *, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
} g_nccl;

bool rccl_load() {
    if (g_nccl.lib) return true;
    for (const char *name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1", "/opt/rocm/lib/librccl.so"})
        if ((g_nccl.lib = dlopen(name, RTLD_NOW | RTLD_LOCAL)) != nullptr) break;
    if (!g_nccl.lib) return false;
    g_nccl.get_unique_id = (decltype(g_nccl.get_unique_id))dlsym(g_nccl.lib, "ncclGetUniqueId");
    g_nccl.comm_init_rank = (decltype(g_nccl.comm_init_rank))dlsym(g_nccl.lib, "ncclCommInitRank");
    g_nccl.all_gather = (decltype(g_nccl.all_gather))dlsym(g_nccl.lib, "ncclAllGather");
    g_nccl.comm_destroy = (decltype(g_nccl.comm_destroy))dlsym(g_nccl.lib, "ncclCommDestroy");
    if (!g_nccl.get_unique_id || !g_nccl.comm_init_rank || !g_nccl.all_gather || !g_nccl.comm_destroy) {
        dlclose(g_nccl.lib);
        g_nccl = RcclApi{};
        return false;
    }
    return true;
}

// collective over the servers: do they all own a GPU of their own (distinct PCI bus ids)?
bool servers_distinct_gpus() {
    char bus[64];
    memset(bus, 0, sizeof bus);
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetPCIBusId(bus, (int)sizeof bus - 1, dev) != hipSuccess)
        snprintf(bus, sizeof bus, "unknown:%d", g_rank);  // no id: treated as a GPU of its own
    std::vector<char> all((size_t)g_S * sizeof bus);
    MPI_Allgather(bus, (int)sizeof bus, MPI_CHAR, all.data(), (int)sizeof bus, MPI_CHAR, g_srvcomm);
    for (int a = 0; a < g_S; a++)
        for (int b = a + 1; b < g_S; b++)
            if (!strncmp(&all[(size_t)a * sizeof bus], &all[(size_t)b * sizeof bus], sizeof bus)) return false;
    return true;
}

// collective over the servers: true when every server loaded RCCL and joined the communicator
bool rccl_init(size_t blob_ints) {
    int me = 0, ok = rccl_load() ? 1 : 0, all = 0;
    MPI_Comm_rank(g_srvcomm, &me);
    MPI_Allreduce(&ok, &all, 1, MPI_INT, MPI_MIN, g_srvcomm);
    if (!all) {
        if (me == 0) fprintf(stderr, "%06d: RCCL: librccl not loadable, host all-gather kept\n", g_rank);
        return false;
    }
    ncclUniqueId id;
    memset(&id, 0, sizeof id);
    if (me == 0 && g_nccl.get_unique_id(&id) != ncclSuccess) ok = 0;
    MPI_Bcast(&id, (int)sizeof id, MPI_BYTE, 0, g_srvcomm);
    MPI_Allreduce(&ok, &all, 1, MPI_INT, MPI_MIN, g_srvcomm);
    if (!all) return false;
    int dev = 0;
    ok = hipGetDevice(&dev) == hipSuccess && hipStreamCreate(&g_rccl.st) == hipSuccess &&
         hipMalloc((void **)&g_rccl.d_blob, sizeof(int) * blob_ints) == hipSuccess &&
         hipMalloc((void **)&g_rccl.d_all, sizeof(int) * blob_ints * (size_t)g_S) == hipSuccess;
    // every server calls the collective init (a failed allocation joins and leaves after)
    if (g_nccl.comm_init_rank(&g_rccl.comm, g_S, id, me) != ncclSuccess) {
        g_rccl.comm = nullptr;
        ok = 0;
    }
    MPI_Allreduce(&ok, &all, 1, MPI_INT, MPI_MIN, g_srvcomm);
    if (!all) {
        if (g_rccl.comm) g_nccl.comm_destroy(g_rccl.comm);
        g_rccl.comm = nullptr;
        if (g_rccl.d_blob) (void)hipFree(g_rccl.d_blob);
        if (g_rccl.d_all) (void)hipFree(g_rccl.d_all);
        if (g_rccl.st) (void)hipStreamDestroy(g_rccl.st);
        g_rccl = Rccl{};
        if (me == 0) fprintf(stderr, "%06d: RCCL: communicator unavailable, host all-gather kept\n", g_rank);
        return false;
    }
    return true;
}

void rccl_fini() {
    if (!g_rccl.comm) return;
    g_nccl.comm_destroy(g_rccl.comm);
    (void)hipFree(g_rccl.d_blob);
    (void)hipFree(g_rccl.d_all);
    (void)hipStreamDestroy(g_rccl.st);
    g_rccl = Rccl{};
}

bool is_server_rank(int r) { return r >= g_master && r < g_master + g_S; }

void emit(void *ctx, int dest, int tag, const void *buf, int nbytes) {
    Loop *L = static_cast<Loop *>(ctx);
    if (is_server_rank(dest) || dest == g_debug) {
        // server-to-server messages never block the loop (the reference's iq, adlb.c:785-803)
        auto *p = new Pending();
        p->buf.assign((const char *)buf, (const char *)buf + nbytes);
        MPI_Isend(p->buf.data(), nbytes, MPI_BYTE, dest, tag, g_all, &p->req);
        L->pend.push_back(p);
    } else {
        // apps have posted (or are about to post) the matching receive
        MPI_Send(buf, nbytes, MPI_BYTE, dest, tag, g_all);
    }
}

void reap(Loop *L, bool wait) {
    size_t k = 0;
    for (Pending *p : L->pend) {
        int flag = 0;
        if (wait) MPI_Wait(&p->req, MPI_STATUS_IGNORE), flag = 1;
        else MPI_Test(&p->req, &flag, MPI_STATUS_IGNORE);
        if (flag) delete p;
        else L->pend[k++] = p;
    }
    L->pend.resize(k);
}

void to_servers(Loop *L, int tag, const void *buf, int nbytes) {
    for (int i = 0; i < g_S; i++)
        if (g_master + i != g_rank) emit(L, g_master + i, tag, buf, nbytes);
}

void check(int rc, const char *what) {
    if (rc < 0) {
        std::string m = std::string(what) + ": " + adlbsrv_last_error();
        die(m.c_str());
    }
}

bool locally_idle(Loop *L) {
    const int active = L->my_apps - L->apps_done;
    return active <= 0 || (adlbsrv_num_parked(g_srv) >= active && adlbsrv_rfr_outstanding(g_srv) == 0);
}

void send_qmstat_row(Loop *L) {
    // update_local_state (adlb.c:3581-3593) only when the row may have changed since the last one
    // (queue events, byte changes of common prefixes, an SS_RFR this server could not serve)
    const long long act = adlbsrv_row_stamp(g_srv);
    if (act == L->row_activity) return;
    L->row_activity = act;
    const int T = (int)g_types.size();
    std::vector<int> row(2 + (size_t)T);
    double nb = 0.0;
    row[0] = L->my_idx;
    check(adlbsrv_my_row(g_srv, &row[1], &nb, row.data() + 2), "qmstat row");
    std::vector<char> msg(sizeof(int) * row.size() + sizeof(double));
    memcpy(msg.data(), row.data(), sizeof(int) * row.size());
    memcpy(msg.data() + sizeof(int) * row.size(), &nb, sizeof nb);
    to_servers(L, TAG_SRV_QMSTAT, msg.data(), (int)msg.size());
}

void declare_exhausted(Loop *L) {
    to_servers(L, TAG_SRV_EXHAUSTED, nullptr, 0);
    check(adlbsrv_exhausted(g_srv), "exhaustion");
}

void exh_round_done(Loop *L) {
    // two consecutive polls with every server idle and no queue event between them
    if (L->exh_all_idle && L->exh_prev_idle && L->exh_sum == L->exh_prev_sum) {
        declare_exhausted(L);
        L->exh_prev_idle = false;
        L->exh_prev_sum = -1;
        return;
    }
    L->exh_prev_idle = L->exh_all_idle;
    L->exh_prev_sum = L->exh_sum;
}

void exh_poll(Loop *L) {
    if (L->exh_wait) return;  // a poll is out
    if (!locally_idle(L)) {
        L->exh_prev_idle = false;
        return;
    }
    L->exh_epoch++;
    L->exh_all_idle = true;
    L->exh_sum = adlbsrv_activity(g_srv);
    if (g_S == 1) {
        exh_round_done(L);
        return;
    }
    int q[2] = {L->exh_epoch, 0};
    L->exh_wait = g_S - 1;
    to_servers(L, TAG_SRV_EXH_QUERY, q, (int)sizeof q);
}

// one steal round: export, all-gather among the servers, settle (no other message in between)
void steal_round(Loop *L) {
    if (g_rccl.comm) {  // device blobs, RCCL all-gather
        const size_t n = L->blob.size();
        check(adlbsrv_group_export_device(g_srv, g_rccl.d_blob), "steal round export (device)");
        if (hipDeviceSynchronize() != hipSuccess ||
            g_nccl.all_gather(g_rccl.d_blob, g_rccl.d_all, n, ncclInt32, g_rccl.comm, g_rccl.st) != ncclSuccess ||
            hipStreamSynchronize(g_rccl.st) != hipSuccess)
            die("steal round: RCCL all-gather failed");
        int settled = 0;
        check(adlbsrv_group_settle_device(g_srv, g_rccl.d_all, g_S, &settled), "steal round settle (device)");
        return;
    }
    check(adlbsrv_group_export(g_srv, L->blob.data()), "steal round export");
    const int n = (int)L->blob.size();
    MPI_Allgather(L->blob.data(), n, MPI_INT, L->blobs.data(), n, MPI_INT, g_srvcomm);
    int settled = 0;
    check(adlbsrv_group_settle(g_srv, L->blobs.data(), g_S, &settled), "steal round settle");
}

template <int N>
void recv_ints(int *b, int src, int tag) {
    MPI_Recv(b, N * (int)sizeof(int), MPI_BYTE, src, tag, g_all, MPI_STATUS_IGNORE);
}

// drain consecutive messages of one tag already waiting (one GPU batch)
void drain(int tag, int first_src, int nints, std::vector<int> &src, std::vector<int> &buf, int cap) {
    src.clear();
    buf.clear();
    auto take = [&](int s) {
        src.push_back(s);
        buf.resize(buf.size() + (size_t)nints);
        MPI_Recv(buf.data() + buf.size() - nints, nints * (int)sizeof(int), MPI_BYTE, s, tag, g_all,
                 MPI_STATUS_IGNORE);
    };
    take(first_src);
    while ((int)src.size() < cap) {
        int flag = 0;
        MPI_Status st;
        MPI_Iprobe(MPI_ANY_SOURCE, tag, g_all, &flag, &st);
        if (!flag) break;
        take(st.MPI_SOURCE);
    }
}

void serve(Loop *L, double max_malloc) {
    const double qm_int = env_d("ADLB_QMSTAT_INTERVAL", 0.1);   // adlb.c:165
    const double exh_int = env_d("ADLB_EXHAUST_INTERVAL", 0.5);  // the reference waits 5 s (adlb.c:490)
    const double ds_int = 10.0;
    const double st_int = env_d("ADLB_STEAL_INTERVAL", 0.01);
    const double st_idle = env_d("ADLB_STEAL_IDLE_INTERVAL", 0.5);
    // ADLB_PUT_BATCH=0: every Put appended on its own (the one-at-a-time path, for comparison)
    const bool put_batching = env_d("ADLB_PUT_BATCH", 1.0) != 0.0;
    const int put_cap = std::max(1, (int)env_d("ADLB_PUT_RUN_CAP", 256));
    const double put_run_s = env_d("ADLB_PUT_RUN_US", 200.0) * 1e-6;
    const int T = (int)g_types.size();
    double t_qm = MPI_Wtime(), t_exh = MPI_Wtime(), t_ds = MPI_Wtime(), t_st = MPI_Wtime();
    std::vector<int> src, buf, one;
    (void)max_malloc;
    while (!L->done) {
        if (!L->pend.empty()) reap(L, false);
        const double t = MPI_Wtime();
        if (g_S > 1 && t - t_qm > qm_int) {
            send_qmstat_row(L);
            t_qm = t;
        }
        if (g_rank == g_master && t - t_exh > exh_int) {
            exh_poll(L);
            t_exh = t;
        }
        // open a steal round when a server asked for one (a parked Reserve has a donor by its
        // qmstat table), at most every st_int; otherwise only every st_idle as a safety net
        if (L->group && g_rank == g_master && ((L->steal_want && t - t_st > st_int) || t - t_st > st_idle)) {
            L->steal_want = false;
            to_servers(L, TAG_SRV_STEAL, nullptr, 0);
            steal_round(L);
            t_st = MPI_Wtime();
        }
        if (g_debug >= 0 && g_rank == g_master && t - t_ds > ds_int) {  // keeps the debug server's watchdog fed
            int b[WIRE_IBUF] = {0};
            emit(L, g_debug, 1031 /* DS_LOG */, b, (int)sizeof b);
            t_ds = t;
        }
        check(adlbsrv_push_tick(g_srv), "push");  // memory-pressure push (adlb.c:509-556)
        int flag = 0;
        MPI_Status st;
        MPI_Iprobe(MPI_ANY_SOURCE, MPI_ANY_TAG, g_all, &flag, &st);
        if (!flag) continue;
        const int from = st.MPI_SOURCE, tag = st.MPI_TAG;
        switch (tag) {
        case TAG_PUT_HDR: {
            // a run of waiting FA_PUT_HDRs: each acked and its payload received in turn
            // (adlb.c:891-962), the appends and rq matches as one engine batch (963-1049).
            // The run holds back its Puts' final acks and the Reserves they match, so it is
            // short: at most put_cap Puts or put_run_s of wall time, and it ends at the first
            // waiting message that is not a Put.  The next header is taken only when an
            // any-tag probe returns it, i.e. it is its source's oldest waiting message, so
            // every app's messages are still handled in the order it sent them.
            int src_put = from, nput = 0;
            const double t_run = MPI_Wtime();
            std::vector<char> p;
            while (true) {
                int h[WIRE_IBUF], need = 0;
                recv_ints<WIRE_IBUF>(h, src_put, TAG_PUT_HDR);
                check(adlbsrv_put_hdr(g_srv, src_put, h, &need), "FA_PUT_HDR");
                if (need) {
                    p.resize((size_t)std::max(h[4], 1));
                    MPI_Recv(p.data(), h[4], MPI_BYTE, src_put, TAG_PUT_MSG, g_all, MPI_STATUS_IGNORE);
                    if (put_batching) check(adlbsrv_put_stage(g_srv, src_put, h, p.data(), h[4]), "FA_PUT_MSG");
                    else check(adlbsrv_put_payload(g_srv, src_put, h, p.data(), h[4]), "FA_PUT_MSG");
                }
                if (++nput >= put_cap || MPI_Wtime() - t_run > put_run_s) break;
                int more = 0;
                MPI_Status pst;
                MPI_Iprobe(MPI_ANY_SOURCE, MPI_ANY_TAG, g_all, &more, &pst);
                if (!more || pst.MPI_TAG != TAG_PUT_HDR) break;
                src_put = pst.MPI_SOURCE;
            }
            check(adlbsrv_put_flush(g_srv), "FA_PUT_MSG (batch)");
            break;
        }
        case TAG_RESERVE:
            drain(TAG_RESERVE, from, WIRE_REQ + 1, src, buf, 1 << 14);
            check(adlbsrv_reserve_batch(g_srv, (int)src.size(), src.data(), buf.data()), "FA_RESERVE");
            break;
        case TAG_GET_RESERVED: {
            drain(TAG_GET_RESERVED, from, WIRE_IBUF, src, buf, 1 << 14);
            one.resize(src.size());
            for (size_t i = 0; i < src.size(); i++) one[i] = buf[i * WIRE_IBUF];
            check(adlbsrv_get_batch(g_srv, (int)src.size(), src.data(), one.data()), "FA_GET_RESERVED");
            break;
        }
        case TAG_INFO_NUM_WORK_UNITS: {
            int b[WIRE_IBUF];
            recv_ints<WIRE_IBUF>(b, from, tag);
            check(adlbsrv_info_num(g_srv, from, b[0]), "FA_INFO_NUM_WORK_UNITS");
            break;
        }
        case TAG_PUT_COMMON_HDR: {
            int h[WIRE_IBUF], need = 0;
            recv_ints<WIRE_IBUF>(h, from, tag);
            check(adlbsrv_put_common_hdr(g_srv, from, h[0], &need), "FA_PUT_COMMON_HDR");
            if (need) {
                std::vector<char> p((size_t)std::max(h[0], 0));
                MPI_Recv(p.data(), h[0], MPI_BYTE, from, TAG_PUT_COMMON_MSG, g_all, MPI_STATUS_IGNORE);
                check(adlbsrv_put_common_payload(g_srv, from, p.data(), h[0]), "FA_PUT_COMMON_MSG");
            }
            break;
        }
        case TAG_PUT_BATCH_DONE: {
            int b[WIRE_IBUF];
            recv_ints<WIRE_IBUF>(b, from, tag);
            check(adlbsrv_batch_done(g_srv, from, b[0], b[1]), "FA_PUT_BATCH_DONE");
            break;
        }
        case TAG_GET_COMMON: {
            int b[WIRE_IBUF];
            recv_ints<WIRE_IBUF>(b, from, tag);
            check(adlbsrv_get_common(g_srv, from, b[0]), "FA_GET_COMMON");
            break;
        }
        case TAG_DID_PUT_AT_REMOTE: {
            int b[WIRE_IBUF];
            recv_ints<WIRE_IBUF>(b, from, tag);
            check(adlbsrv_did_put_at_remote(g_srv, b[0], b[1], b[2]), "FA_DID_PUT_AT_REMOTE");
            break;
        }
        case TAG_NO_MORE_WORK: {
            MPI_Recv(nullptr, 0, MPI_BYTE, from, tag, g_all, MPI_STATUS_IGNORE);
            const int fresh = adlbsrv_no_more_work(g_srv);
            check(fresh, "FA_NO_MORE_WORK");
            if (fresh == 1) to_servers(L, TAG_SS_NO_MORE_WORK, nullptr, 0);
            break;
        }
        case TAG_SS_NO_MORE_WORK:
            MPI_Recv(nullptr, 0, MPI_BYTE, from, tag, g_all, MPI_STATUS_IGNORE);
            check(adlbsrv_no_more_work(g_srv), "SS_NO_MORE_WORK");
            break;
        case TAG_LOCAL_APP_DONE:
            MPI_Recv(nullptr, 0, MPI_BYTE, from, tag, g_all, MPI_STATUS_IGNORE);
            if (++L->apps_done == L->my_apps) {
                if (g_rank == g_master) {
                    if (++L->servers_done == g_S) L->done = true;
                } else {
                    emit(L, g_master, TAG_SRV_DONE, nullptr, 0);
                }
            }
            break;
        case TAG_SRV_DONE:
            MPI_Recv(nullptr, 0, MPI_BYTE, from, tag, g_all, MPI_STATUS_IGNORE);
            if (++L->servers_done == g_S) L->done = true;
            break;
        case TAG_SRV_END:
            MPI_Recv(nullptr, 0, MPI_BYTE, from, tag, g_all, MPI_STATUS_IGNORE);
            L->done = true;
            break;
        case TAG_SRV_STEAL:
            MPI_Recv(nullptr, 0, MPI_BYTE, from, tag, g_all, MPI_STATUS_IGNORE);
            if (L->group) steal_round(L);
            break;
        case TAG_SRV_STEAL_WANT:
            MPI_Recv(nullptr, 0, MPI_BYTE, from, tag, g_all, MPI_STATUS_IGNORE);
            L->steal_want = true;
            break;
        case TAG_SRV_QMSTAT: {
            std::vector<char> m(sizeof(int) * (2 + (size_t)T) + sizeof(double));
            MPI_Recv(m.data(), (int)m.size(), MPI_BYTE, from, tag, g_all, MPI_STATUS_IGNORE);
            int idx;
            memcpy(&idx, m.data(), sizeof idx);
            if (idx >= 0 && idx < g_S) {
                memcpy(&L->qlen[(size_t)idx], m.data() + sizeof(int), sizeof(int));
                memcpy(L->hi.data() + (size_t)idx * T, m.data() + 2 * sizeof(int), sizeof(int) * (size_t)T);
                memcpy(&L->nbytes[(size_t)idx], m.data() + sizeof(int) * (2 + (size_t)T), sizeof(double));
                check(adlbsrv_qmstat(g_srv, L->qlen.data(), L->nbytes.data(), L->hi.data()), "SS_QMSTAT");
            }
            break;
        }
        case TAG_SS_RFR: {
            int b[WIRE_RFR];
            recv_ints<WIRE_RFR>(b, from, tag);
            check(adlbsrv_rfr(g_srv, from, b), "SS_RFR");
            break;
        }
        case TAG_SS_RFR_RESP: {
            int b[WIRE_RFR];
            recv_ints<WIRE_RFR>(b, from, tag);
            check(adlbsrv_rfr_resp(g_srv, from, b), "SS_RFR_RESP");
            break;
        }
        case TAG_SS_UNRESERVE: {
            int b[WIRE_IBUF];
            recv_ints<WIRE_IBUF>(b, from, tag);
            check(adlbsrv_unreserve(g_srv, from, b), "SS_UNRESERVE");
            break;
        }
        case TAG_SS_PUSH_QUERY: {
            double d[WIRE_IBUF];
            MPI_Recv(d, (int)sizeof d, MPI_BYTE, from, tag, g_all, MPI_STATUS_IGNORE);
            check(adlbsrv_push_query(g_srv, from, d), "SS_PUSH_QUERY");
            break;
        }
        case TAG_SS_PUSH_QUERY_RESP: {
            double d[WIRE_IBUF];
            MPI_Recv(d, (int)sizeof d, MPI_BYTE, from, tag, g_all, MPI_STATUS_IGNORE);
            check(adlbsrv_push_query_resp(g_srv, from, d), "SS_PUSH_QUERY_RESP");
            break;
        }
        case TAG_SS_PUSH_HDR: {  // the payload follows as SS_PUSH_WORK (adlb.c:2243-2244)
            int b[WIRE_IBUF];
            recv_ints<WIRE_IBUF>(b, from, tag);
            const int len = adlbsrv_push_len(g_srv, b[0]);
            if (len < 0) die("SS_PUSH_HDR for a unit this server does not hold");
            std::vector<char> p((size_t)std::max(len, 1));
            MPI_Recv(p.data(), len, MPI_BYTE, from, TAG_SS_PUSH_WORK, g_all, MPI_STATUS_IGNORE);
            check(adlbsrv_push_hdr(g_srv, from, b, p.data(), len), "SS_PUSH_HDR");
            break;
        }
        case TAG_SS_PUSH_DEL: {
            int b[WIRE_IBUF];
            recv_ints<WIRE_IBUF>(b, from, tag);
            check(adlbsrv_push_del(g_srv, from, b), "SS_PUSH_DEL");
            break;
        }
        case TAG_SS_MOVING_TARGETED_WORK: {
            int b[WIRE_IBUF];
            recv_ints<WIRE_IBUF>(b, from, tag);
            check(adlbsrv_moving_targeted(g_srv, from, b), "SS_MOVING_TARGETED_WORK");
            break;
        }
        case TAG_SRV_EXH_QUERY: {
            int q[2];
            MPI_Recv(q, (int)sizeof q, MPI_BYTE, from, tag, g_all, MPI_STATUS_IGNORE);
            long long r[3] = {q[0], locally_idle(L) ? 1 : 0, adlbsrv_activity(g_srv)};
            emit(L, from, TAG_SRV_EXH_REPLY, r, (int)sizeof r);
            break;
        }
        case TAG_SRV_EXH_REPLY: {
            long long r[3];
            MPI_Recv(r, (int)sizeof r, MPI_BYTE, from, tag, g_all, MPI_STATUS_IGNORE);
            if (r[0] == L->exh_epoch && L->exh_wait > 0) {
                L->exh_all_idle = L->exh_all_idle && r[1];
                L->exh_sum += r[2];
                if (--L->exh_wait == 0) exh_round_done(L);
            }
            break;
        }
        case TAG_SRV_EXHAUSTED:
            MPI_Recv(nullptr, 0, MPI_BYTE, from, tag, g_all, MPI_STATUS_IGNORE);
            check(adlbsrv_exhausted(g_srv), "SS_DONE_BY_EXHAUSTION");
            break;
        case TAG_FA_ABORT:
        case TAG_SRV_ABORT: {
            int b[WIRE_IBUF] = {-1};
            MPI_Recv(b, (int)sizeof b, MPI_BYTE, from, tag, g_all, MPI_STATUS_IGNORE);
            fprintf(stderr, "%06d: ** ADLB abort %d requested by rank %d\n", g_rank, b[0], from);
            MPI_Abort(MPI_COMM_WORLD, b[0]);
            break;
        }
        default: {
            int n = 0;
            MPI_Get_count(&st, MPI_BYTE, &n);
            std::vector<char> junk((size_t)std::max(n, 1));
            MPI_Recv(junk.data(), n, MPI_BYTE, from, tag, g_all, MPI_STATUS_IGNORE);
            fprintf(stderr, "%06d: ** adlb_server: unexpected tag %d from %d\n", g_rank, tag, from);
        }
        }
    }
    if (g_rank == g_master) {  // SS_END_LOOP_2 / DS_END (adlb.c:1524-1542, 1771-1779)
        to_servers(L, TAG_SRV_END, nullptr, 0);
        if (g_debug >= 0) emit(L, g_debug, TAG_DS_END, nullptr, 0);
    }
    reap(L, true);
}

}  // namespace

extern "C" {

// ------------------------------------------------------------------ setup
int ADLBP_Init(int nservers, int use_debug_server, int aprintf_flag, int ntypes, int *types, int *am_server,
               int *am_debug_server, MPI_Comm *app_comm) {
    int flag = 0;
    MPI_Initialized(&flag);
    if (!flag) {
        fprintf(stderr, "** ADLB_Init: MPI is not initialised\n");
        return ADLB_ERROR;
    }
    MPI_Comm_size(MPI_COMM_WORLD, &g_world);
    MPI_Comm_rank(MPI_COMM_WORLD, &g_rank);
    g_t0 = MPI_Wtime();
    g_dbgprintf = aprintf_flag;
    g_types.assign(types, types + ntypes);
    g_S = nservers;
    g_debug = use_debug_server ? g_world - 1 : -1;
    g_A = g_world - nservers - (use_debug_server ? 1 : 0);  // adlb.c:240-252
    g_master = g_A;
    if (nservers < 1 || g_A < 1) {
        fprintf(stderr, "** ADLB_Init: %d ranks cannot hold %d server(s)%s and an app\n", g_world, nservers,
                use_debug_server ? " + debug server" : "");
        return ADLB_ERROR;
    }
    if (g_rank < g_A) {  // adlb.c:254-259
        *am_server = 0;
        *am_debug_server = 0;
        MPI_Comm_split(MPI_COMM_WORLD, 0, g_rank, app_comm);
        g_home = g_A + g_rank % g_S;
    } else if (g_rank == g_debug) {
        *am_server = 0;
        *am_debug_server = 1;
        MPI_Comm dc;
        MPI_Comm_split(MPI_COMM_WORLD, 2, 0, &dc);
        MPI_Comm_free(&dc);
        g_is_debug = true;
    } else {
        *am_server = 1;
        *am_debug_server = 0;
        MPI_Comm_split(MPI_COMM_WORLD, 1, g_rank - g_A, &g_srvcomm);
        g_is_server = true;
    }
    MPI_Comm_dup(MPI_COMM_WORLD, &g_all);
    g_next_put = g_home;  // adlb.c:377
    g_common_len = 0, g_common_server = -1, g_common_seqno = -1, g_common_refcnt = 0, g_in_batch = 0;
    return ADLB_SUCCESS;
}

int ADLBP_Server(double hi_malloc, double periodic_logging_time) {
    (void)periodic_logging_time;
    if (!g_is_server) return ADLB_ERROR;
    Loop L;
    L.my_idx = g_rank - g_master;
    for (int i = 0; i < g_A; i++) L.my_apps += (g_A + i % g_S) == g_rank;
    const int T = (int)g_types.size();
    L.qlen.assign((size_t)g_S, 0);
    L.nbytes.assign((size_t)g_S, 0.0);
    L.hi.assign((size_t)g_S * T, ADLB_LOWEST_PRIO);
    const char *dv = getenv("ADLB_DEVICE");
    const int device = dv && *dv ? atoi(dv) : -1;
    if (adlbsrv_create(&g_srv, T, g_types.data(), g_A, g_S, g_rank, hi_malloc, device, emit, &L) < 0) {
        std::string m = std::string("server create: ") + adlbsrv_last_error();
        die(m.c_str());
    }
    // steal group: every server on one node (or forced by ADLB_STEAL_GROUP); the
    // decision is collective so that all servers run the rounds or none does
    int want = 0;
    if (g_S > 1) {
        MPI_Comm node;
        int nn = 0;
        MPI_Comm_split_type(g_srvcomm, MPI_COMM_TYPE_SHARED, 0, MPI_INFO_NULL, &node);
        MPI_Comm_size(node, &nn);
        MPI_Comm_free(&node);
        const char *sg = getenv("ADLB_STEAL_GROUP");
        want = sg && *sg ? atoi(sg) != 0 : nn == g_S;
        // the merge's type sets are 64-bit masks (adlbq_steal_group_export): a server of more
        // types keeps the reference's SS_RFR steals (adlb.c:1280-1308), whatever was asked for.
        // Every server declared the same types (ADLB_Init), so this agrees on all of them.
        if (T > ADLBQ_MAX_TYPES) want = 0;
    } else {
        // one server: a steal group only when asked for (the round path exercised, nothing to steal)
        const char *sg = getenv("ADLB_STEAL_GROUP");
        want = sg && *sg && atoi(sg) != 0 && T <= ADLBQ_MAX_TYPES;
    }
    int all_want = 0;
    MPI_Allreduce(&want, &all_want, 1, MPI_INT, MPI_MIN, g_srvcomm);
    if (all_want) {
        const int k = std::max(1, (int)env_d("ADLB_STEAL_K", 64)), rqcap = std::max(1, (int)env_d("ADLB_STEAL_RQCAP", 1024));
        check(adlbsrv_group_create(g_srv, k, rqcap), "steal group");
        L.group = true;
        L.blob.assign((size_t)adlbsrv_group_blob_ints(g_srv), 0);
        L.blobs.assign(L.blob.size() * (size_t)g_S, 0);
        // the transport: RCCL when every server owns a GPU of its own (or when forced), else MPI_Allgather
        const char *rv = getenv("ADLB_STEAL_RCCL");
        const int mode = rv && *rv ? atoi(rv) : -1;  // -1: automatic
        const bool distinct = servers_distinct_gpus();  // collective
        int try_rccl = mode == 0 ? 0 : (mode > 0 || distinct) ? 1 : 0, all_try = 0;
        MPI_Allreduce(&try_rccl, &all_try, 1, MPI_INT, MPI_MIN, g_srvcomm);
        const bool on = all_try && rccl_init(L.blob.size());  // collective
        if (getenv("ADLB_STEAL_REPORT")) {
            if (on) fprintf(stderr, "%06d: RCCL all-gather of the steal blobs on (%d servers)\n", g_rank, g_S);
            fprintf(stderr, "%06d: steal transport: %s\n", g_rank,
                    on ? "rccl" : mode == 0 ? "mpi (ADLB_STEAL_RCCL=0)" : !distinct && mode < 0 ? "mpi (servers share a GPU)"
                                                                                    : "mpi (RCCL unavailable)");
        }
    }
    g_loop = &L;
    if (L.my_apps == 0 && g_rank != g_master) emit(&L, g_master, TAG_SRV_DONE, nullptr, 0);
    if (L.my_apps == 0 && g_rank == g_master && ++L.servers_done == g_S) L.done = true;
    serve(&L, hi_malloc);
    if (L.group && getenv("ADLB_STEAL_REPORT"))
        fprintf(stderr, "%06d: steal group: %lld rounds, %lld Reserves settled by the merge, %lld SS_RFR sent\n", g_rank,
                adlbsrv_group_stat(g_srv, 0), adlbsrv_group_stat(g_srv, 1), adlbsrv_group_stat(g_srv, 2));
    rccl_fini();
    g_loop = nullptr;
    return ADLB_SUCCESS;
}

int ADLBP_Debug_server(double timeout) {
    // a watchdog: ends on DS_END, aborts the job when nothing arrived for timeout s (adlb.c:2528-2636)
    double last = MPI_Wtime();
    while (true) {
        if (MPI_Wtime() - last > timeout) {
            fprintf(stderr, "%06d: ** debug_server: no messages for %.0f s; aborting\n", g_rank, timeout);
            MPI_Abort(MPI_COMM_WORLD, -1);
        }
        int flag = 0;
        MPI_Status st;
        MPI_Iprobe(MPI_ANY_SOURCE, MPI_ANY_TAG, g_all, &flag, &st);
        if (!flag) {
            usleep(1000);
            continue;
        }
        int n = 0;
        MPI_Get_count(&st, MPI_BYTE, &n);
        std::vector<char> b((size_t)std::max(n, 1));
        MPI_Recv(b.data(), n, MPI_BYTE, st.MPI_SOURCE, st.MPI_TAG, g_all, MPI_STATUS_IGNORE);
        last = MPI_Wtime();
        if (st.MPI_TAG == TAG_DS_END || st.MPI_TAG == TAG_FA_ABORT) break;
    }
    return ADLB_SUCCESS;
}

int ADLBP_Finalize(void) {
    int flag = 0;
    MPI_Finalized(&flag);
    if (flag) {
        printf("** OOPS; you should not call MPI_Finalize before ADLB_Finalize\n");
        return ADLB_ERROR;
    }
    if (g_is_server) {
        adlbsrv_destroy(g_srv);
        g_srv = nullptr;
    } else if (!g_is_debug && g_home >= 0) {
        int dummy = 0;
        MPI_Ssend(&dummy, 0, MPI_INT, g_home, TAG_LOCAL_APP_DONE, g_all);  // adlb.c:3158
    }
    if (g_srvcomm != MPI_COMM_NULL) MPI_Comm_free(&g_srvcomm);
    if (g_all != MPI_COMM_NULL) MPI_Comm_free(&g_all);
    return ADLB_SUCCESS;
}

int ADLBP_Abort(int code) {
    fprintf(stderr, "%06d: ** ADLB_Abort(%d): invoking MPI_Abort\n", g_rank, code);
    fflush(stderr);
    MPI_Abort(MPI_COMM_WORLD, code);
    return -1;
}

// ------------------------------------------------------------------ app side
int ADLBP_Put(void *work_buf, int work_len, int target_rank, int answer_rank, int work_type, int work_prio) {
    if (work_type < -1 || !type_ok(work_type)) {  // adlb.c:2762-2766
        fprintf(stderr, "%06d: ** invalid work_type %d to ADLB_Put\n", g_rank, work_type);
        ADLBP_Abort(-1);
    }
    int to = target_rank >= 0 ? g_A + target_rank % g_S : next_put_server();
    const int home = to;
    int attempts = 0, sleeps = 0, others_may_have_space = 1;
    int ack[WIRE_IBUF];
    while (true) {  // the rejection walk of adlb.c:2780-2841
        if (attempts && attempts % g_S == 0) {
            if (attempts >= 2 * g_S && !others_may_have_space) {
                sleep(1);
                if (++sleeps > 1000) return ADLB_PUT_REJECTED;
            }
            others_may_have_space = 0;
        }
        attempts++;
        int h[WIRE_IBUF] = {work_type, work_prio,      answer_rank,     target_rank,      work_len, home,
                            g_in_batch, g_common_len, g_common_server, g_common_seqno, 0,        0};
        MPI_Request r;
        MPI_Irecv(ack, WIRE_IBUF, MPI_INT, to, TAG_ACK_AND_RC, g_all, &r);
        MPI_Send(h, WIRE_IBUF, MPI_INT, to, TAG_PUT_HDR, g_all);
        MPI_Wait(&r, MPI_STATUS_IGNORE);
        if (ack[0] == ADLB_NO_MORE_WORK || ack[0] == ADLB_DONE_BY_EXHAUSTION) return ack[0];
        if (ack[0] == ADLB_PUT_REJECTED) {
            if (ack[1] >= 0) others_may_have_space = 1;
            to = next_put_server();
            continue;
        }
        if (ack[0] < 0) return ack[0];
        MPI_Send(work_buf, work_len, MPI_BYTE, to, TAG_PUT_MSG, g_all);
        MPI_Recv(ack, WIRE_IBUF, MPI_INT, to, TAG_ACK_AND_RC, g_all, MPI_STATUS_IGNORE);
        if (target_rank >= 0 && home != to) {  // adlb.c:2845-2852
            int b[WIRE_IBUF] = {work_type, target_rank, to};
            MPI_Send(b, WIRE_IBUF, MPI_INT, home, TAG_DID_PUT_AT_REMOTE, g_all);
        }
        if (g_common_len > 0) g_common_refcnt++;
        return ack[0] < 0 ? ack[0] : ADLB_SUCCESS;
    }
}

int adlbp_Reserve(int *req_types, int *work_type, int *work_prio, int *work_handle, int *work_len,
                  int *answer_rank, int hang_flag) {
    for (int i = 0; i < WIRE_REQ; i++) {  // adlb.c:2893-2902
        if (req_types[i] == -1) break;
        if (req_types[i] < -1 || !type_ok(req_types[i])) {
            fprintf(stderr, "%06d: ** invalid req_type %d to adlb reserve\n", g_rank, req_types[i]);
            ADLBP_Abort(-1);
        }
    }
    int b[WIRE_REQ + 1];
    b[0] = hang_flag;
    b[1] = req_types[0];
    for (int i = 1; i < WIRE_REQ; i++) {  // after the first -1 everything is padding (adlb.c:2905-2916)
        if (req_types[0] == -1 || req_types[i] == -1) {
            for (int j = i; j < WIRE_REQ; j++) b[j + 1] = -2;
            break;
        }
        b[i + 1] = req_types[i];
    }
    int info[WIRE_IBUF];
    MPI_Request r;
    MPI_Irecv(info, WIRE_IBUF, MPI_INT, g_home, TAG_RESERVE_RESP, g_all, &r);
    MPI_Send(b, WIRE_REQ + 1, MPI_INT, g_home, TAG_RESERVE, g_all);
    MPI_Wait(&r, MPI_STATUS_IGNORE);
    if (info[0] == WIRE_NO_CURR_WORK) return ADLB_NO_CURRENT_WORK;
    if (info[0] < 0) return info[0];
    *work_type = info[1];
    *work_prio = info[2];
    *work_len = info[3];
    *answer_rank = info[4];
    work_handle[0] = info[5];  // wqseqno
    work_handle[1] = info[6];  // server holding the unit
    work_handle[2] = info[7];  // common_len
    if (info[7] > 0) *work_len += info[7];
    work_handle[3] = info[8];  // common server
    work_handle[4] = info[9];  // common seqno
    return ADLB_SUCCESS;
}

int ADLBP_Reserve(int *req_types, int *work_type, int *work_prio, int *work_handle, int *work_len,
                  int *answer_rank) {
    return adlbp_Reserve(req_types, work_type, work_prio, work_handle, work_len, answer_rank, 1);
}

int ADLBP_Ireserve(int *req_types, int *work_type, int *work_prio, int *work_handle, int *work_len,
                   int *answer_rank) {
    return adlbp_Reserve(req_types, work_type, work_prio, work_handle, work_len, answer_rank, 0);
}

int adlbp_Get_reserved_timed(void *work_buf, int *work_handle, double *queued_time) {
    const int commlen = work_handle[2];
    if (commlen > 0) {  // the common prefix first (adlb.c:2985-2993)
        int b[WIRE_IBUF] = {work_handle[4]};
        MPI_Send(b, WIRE_IBUF, MPI_INT, work_handle[3], TAG_GET_COMMON, g_all);
        MPI_Recv(work_buf, commlen, MPI_BYTE, work_handle[3], TAG_GET_COMMON_RESP, g_all, MPI_STATUS_IGNORE);
    }
    const int from = work_handle[1];
    int b[WIRE_IBUF] = {work_handle[0]};
    double d[WIRE_IBUF];
    MPI_Request r;
    MPI_Irecv(d, WIRE_IBUF, MPI_DOUBLE, from, TAG_ACK_AND_RC, g_all, &r);
    MPI_Send(b, WIRE_IBUF, MPI_INT, from, TAG_GET_RESERVED, g_all);
    MPI_Wait(&r, MPI_STATUS_IGNORE);
    if ((int)d[0] < 0) return (int)d[0];
    const int len = (int)d[1];
    MPI_Recv((char *)work_buf + (commlen > 0 ? commlen : 0), len, MPI_BYTE, from, TAG_GET_RESERVED_RESP, g_all,
             MPI_STATUS_IGNORE);
    if (queued_time) *queued_time = d[2];
    return ADLB_SUCCESS;
}

int ADLBP_Get_reserved(void *work_buf, int *work_handle) {
    return adlbp_Get_reserved_timed(work_buf, work_handle, nullptr);
}

int ADLBP_Get_reserved_timed(void *work_buf, int *work_handle, double *queued_time) {
    return adlbp_Get_reserved_timed(work_buf, work_handle, queued_time);
}

int ADLBP_Begin_batch_put(void *common_buf, int len_common) {
    g_in_batch = 1;
    if (len_common <= 0) return ADLB_SUCCESS;
    int to = next_put_server(), attempts = 0, sleeps = 0, others_may_have_space = 1;
    int ack[WIRE_IBUF];
    while (true) {  // adlb.c:2659-2727
        if (attempts && attempts % g_S == 0) {
            if (attempts >= 2 * g_S && !others_may_have_space) {
                sleep(1);
                if (++sleeps > 1000) return ADLB_PUT_REJECTED;
            }
            others_may_have_space = 0;
        }
        attempts++;
        int h[WIRE_IBUF] = {len_common};
        MPI_Ssend(h, WIRE_IBUF, MPI_INT, to, TAG_PUT_COMMON_HDR, g_all);
        MPI_Recv(ack, WIRE_IBUF, MPI_INT, to, TAG_ACK_AND_RC, g_all, MPI_STATUS_IGNORE);
        if (ack[0] == ADLB_NO_MORE_WORK || ack[0] == ADLB_DONE_BY_EXHAUSTION) return ack[0];
        if (ack[0] == ADLB_PUT_REJECTED) {
            if (ack[1] >= 0) others_may_have_space = 1;
            to = next_put_server();
            continue;
        }
        if (ack[0] < 0) return ack[0];
        MPI_Ssend(common_buf, len_common, MPI_BYTE, to, TAG_PUT_COMMON_MSG, g_all);
        MPI_Recv(ack, WIRE_IBUF, MPI_INT, to, TAG_ACK_AND_RC, g_all, MPI_STATUS_IGNORE);
        if (ack[0] < 0) return ack[0];
        g_common_len = len_common;
        g_common_refcnt = 0;
        g_common_server = to;
        g_common_seqno = ack[1];
        return ADLB_SUCCESS;
    }
}

int ADLBP_End_batch_put(void) {
    int rc = ADLB_SUCCESS;
    if (g_common_server >= 0) {  // adlb.c:2737-2743
        int b[WIRE_IBUF] = {g_common_seqno, g_common_refcnt};
        MPI_Ssend(b, WIRE_IBUF, MPI_INT, g_common_server, TAG_PUT_BATCH_DONE, g_all);
        MPI_Recv(b, WIRE_IBUF, MPI_INT, g_common_server, TAG_ACK_AND_RC, g_all, MPI_STATUS_IGNORE);
        rc = b[0];
    }
    g_common_len = 0, g_common_refcnt = 0, g_common_server = -1, g_common_seqno = -1, g_in_batch = 0;
    return rc;
}

int ADLBP_Set_problem_done(void) {
    int dummy = 0;
    MPI_Ssend(&dummy, 0, MPI_BYTE, g_home, TAG_NO_MORE_WORK, g_all);  // adlb.c:3059-3063
    return ADLB_SUCCESS;
}

int ADLBP_Set_no_more_work(void) { return ADLBP_Set_problem_done(); }

int ADLBP_Info_num_work_units(int work_type, int *max_prio, int *num_max_prio_type, int *num_type) {
    if (!type_ok(work_type)) {  // adlb.c:3033-3037
        fprintf(stderr, "%06d: ** aborting: INVALID TYPE %d\n", g_rank, work_type);
        ADLBP_Abort(-1);
    }
    int b[WIRE_IBUF] = {work_type};
    MPI_Ssend(b, WIRE_IBUF, MPI_INT, g_home, TAG_INFO_NUM_WORK_UNITS, g_all);
    MPI_Recv(b, WIRE_IBUF, MPI_INT, g_home, TAG_ACK_AND_RC, g_all, MPI_STATUS_IGNORE);
    *max_prio = b[0];
    *num_max_prio_type = b[1];
    *num_type = b[2];
    return b[3];  // 0, or ADLB_NO_MORE_WORK (adlb.c:3044)
}

int ADLBP_Info_get(int key, double *val) {
    if (key < ADLB_INFO_MALLOC_HWM || key > ADLB_INFO_MAX_WQ_COUNT) return ADLB_ERROR;
    if (g_srv) return adlbsrv_info_get(g_srv, key, val) < 0 ? ADLB_ERROR : ADLB_SUCCESS;
    *val = 0.0;  // an app keeps none of the server statistics
    return ADLB_SUCCESS;
}

void adlbp_dbgprintf(int flag, int linenum, char *fmt, ...) {
    if (!g_dbgprintf || !flag) return;
    va_list ap;
    va_start(ap, fmt);
    char *s = nullptr;
    if (vasprintf(&s, fmt, ap) < 0) s = nullptr;
    va_end(ap);
    if (!s) return;
    fprintf(stderr, "%06d: %4d: %f:  %s", g_rank, linenum, MPI_Wtime() - g_t0, s);
    fflush(stderr);
    free(s);
}

// the reference's allocation helpers (adlb.c:3419-3474), exported for code that calls them
static double g_dm_curr = 0.0;
void *pmalloc(int nbytes, const char *funcname, int linenum) {
    (void)funcname, (void)linenum;
    void *p = malloc((size_t)std::max(nbytes, 1));
    if (p) g_dm_curr += nbytes;
    return p;
}
void *dmalloc(int nbytes, const char *funcname, int linenum) {
    void *p = pmalloc(nbytes, funcname, linenum);
    if (!p) {
        fprintf(stderr, "%06d: ** dmalloc of %d bytes failed in %s:%d\n", g_rank, nbytes, funcname, linenum);
        MPI_Abort(MPI_COMM_WORLD, -1);
    }
    return p;
}
void dfree(void *ptr, int nbytes, const char *funcname, int linenum) {
    (void)funcname, (void)linenum;
    free(ptr);
    g_dm_curr -= nbytes;
}

int adlbp_Probe(int dest, int tag, MPI_Comm comm, MPI_Status *status) { return MPI_Probe(dest, tag, comm, status); }
int adlb_Probe(int dest, int tag, MPI_Comm comm, MPI_Status *status) { return adlbp_Probe(dest, tag, comm, status); }

// ------------------------------------------------------------------ ADLB_* -> ADLBP_* (adlb_prof.c)
int ADLB_Init(int a, int b, int c, int d, int *e, int *f, int *g, MPI_Comm *h) { return ADLBP_Init(a, b, c, d, e, f, g, h); }
int ADLB_Server(double a, double b) { return ADLBP_Server(a, b); }
int ADLB_Debug_server(double a) { return ADLBP_Debug_server(a); }
int ADLB_Put(void *a, int b, int c, int d, int e, int f) { return ADLBP_Put(a, b, c, d, e, f); }
int ADLB_Reserve(int *a, int *b, int *c, int *d, int *e, int *f) { return ADLBP_Reserve(a, b, c, d, e, f); }
int ADLB_Ireserve(int *a, int *b, int *c, int *d, int *e, int *f) { return ADLBP_Ireserve(a, b, c, d, e, f); }
int ADLB_Get_reserved(void *a, int *b) { return ADLBP_Get_reserved(a, b); }
int ADLB_Get_reserved_timed(void *a, int *b, double *c) { return ADLBP_Get_reserved_timed(a, b, c); }
int ADLB_Begin_batch_put(void *a, int b) { return ADLBP_Begin_batch_put(a, b); }
int ADLB_End_batch_put(void) { return ADLBP_End_batch_put(); }
int ADLB_Begin_batch_put_2(void *a, int b) { return ADLBP_Begin_batch_put(a, b); }
int ADLB_End_batch_put_2(void) { return ADLBP_End_batch_put(); }
int ADLB_Set_problem_done(void) { return ADLBP_Set_problem_done(); }
int ADLB_Set_no_more_work(void) { return ADLBP_Set_no_more_work(); }
int ADLB_Info_get(int a, double *b) { return ADLBP_Info_get(a, b); }
int ADLB_Info_num_work_units(int a, int *b, int *c, int *d) { return ADLBP_Info_num_work_units(a, b, c, d); }
int ADLB_Finalize(void) { return ADLBP_Finalize(); }
int ADLB_Abort(int a) { return ADLBP_Abort(a); }

}  // extern "C"
