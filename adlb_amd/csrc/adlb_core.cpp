// adlb_core.cpp -- the ADLB server's message handlers over the adlbq engine.
//
// Each handler restates one branch of the reference server loop
// (ADLBP_Server, src/adlb.c:382-2500) with the queue work replaced by adlbq
// calls (GPU) and the replies emitted in the reference's order.  Host-side
// state: unit payloads and put timestamps (wqseqno -> bytes), common prefixes
// (cq), the parked Reserves' type vectors (for the SS_RFR buffers), and the
// counters behind ADLB_Info_get.
#include "adlb_core.h"

#include <chrono>
#include <climits>
#include <cstring>
#include <map>
#include <string>
#include <tuple>
#include <unordered_map>
#include <vector>

#include "adlb_wire.h"
#include "adlbq.h"

namespace {

thread_local std::string g_err;

int fail(const std::string &m) {
    g_err = m;
    return -1;
}

double now() {
    using namespace std::chrono;
    return duration<double>(steady_clock::now().time_since_epoch()).count();
}

struct Unit {
    std::vector<char> buf;
    double t = 0.0;  // ws->time_stamp (adlb.c:972)
    int fields[ADLBQ_PUT_INTS];  // the Put's record (a push re-sends it, adlb.c:533-543)
    bool has_fields = false;
};

struct Common {
    std::vector<char> buf;
    int refcnt = -1;  // unknown until FA_PUT_BATCH_DONE (adlb.c:1144)
    int ngets = 0;
};

struct Held {  // a unit accepted by SS_PUSH_QUERY, until SS_PUSH_HDR / SS_PUSH_DEL
    int type = 0, prio = 0, len = 0, answer = -1, target = -1, home = -1, clen = 0, csrv = -1, cseq = -1;
    double t = 0.0;  // the pusher's time stamp (dbls_info_buf[4], adlb.c:2150)
};

struct Staged {  // an accepted Put whose payload arrived, not yet appended
    int src = -1;
    int u[ADLBQ_PUT_INTS];
    int hdr[WIRE_IBUF];
    std::vector<char> buf;
};

struct Parked {
    int rank = -1;
    int types[WIRE_REQ];
    double t = 0.0;
};

}  // namespace

struct adlbsrv {
    adlbq_server *q = nullptr;
    int T = 0, A = 0, S = 1, me = 0, master = 0;
    double max_malloc = 0.0;
    adlbsrv_emit_fn emit = nullptr;
    void *ctx = nullptr;
    bool nmw = false;
    std::unordered_map<int, Unit> units;
    std::unordered_map<int, Common> cq;
    int next_cq = 1;
    std::unordered_map<int, Parked> parked;  // rqseqno -> parked Reserve
    int rfr_out = 0;
    long long activity = 0;
    // ADLB_Info_get counters (adlb.c:3072-3141)
    long long num_reserves = 0, num_put_on_rq = 0, num_rejected = 0, n_rq_timed = 0;
    double time_on_rq = 0.0;
    std::vector<char> first_time_on_rq;
    std::vector<int> reqs, resp, pairs, out5, crem, rqx;
    // push protocol (adlb.c:93, 493, 509-556)
    bool push_out = false;
    long long push_seen = -1;  // state stamp of the last loop-top check that sent nothing
    long long npushed_from = 0, npushed_to = 0, table_events = 0;
    long long row_events = 0;  // changes to this server's qmstat row that are not queue activity (bytes, RFR misses)
    std::unordered_map<int, Held> held;
    // steal group (adlbsrv_group_*): the node's servers settle their parked
    // Reserves in export -> all-gather -> merge rounds instead of SS_RFR round
    // trips; an SS_RFR still goes where the donor may be a tq entry (targeted
    // units put away from their home server), which a round never exports.
    adlbq_steal_group *grp = nullptr;
    std::map<std::tuple<int, int, int>, int> tq;  // (app rank, type, server) -> units: the engine's tq, mirrored
    long long grp_rounds = 0, grp_settled = 0, rfr_sent = 0;
    bool want_sent = false;  // a TAG_SRV_STEAL_WANT went to the master since the last round
    // staged Puts (adlbsrv_put_stage / _flush): payloads in arrival order, the
    // exact byte count when staging began and the bytes the staged Puts add
    std::vector<Staged> staged;
    double staged_base = 0.0, staged_add = 0.0;
    std::vector<int> su, so;
    std::vector<int> grp_rows;

    int rc(int r, const char *what) {
        if (r) g_err = std::string(what) + ": " + adlbq_last_error();
        return r ? -1 : 0;
    }
    void send(int dest, int tag, const void *b, int n) { emit(ctx, dest, tag, b, n); }
    void send_ints(int dest, int tag, const int *v, int n) { send(dest, tag, v, (int)sizeof(int) * n); }
    void send_rc(int dest, int tag, int code) {
        int b[WIRE_IBUF] = {code};
        send_ints(dest, tag, b, WIRE_IBUF);
    }
    bool tq_has(int rank, int server) const {
        auto it = tq.lower_bound(std::make_tuple(rank, INT_MIN, INT_MIN));
        for (; it != tq.end() && std::get<0>(it->first) == rank; ++it)
            if (std::get<2>(it->first) == server && it->second > 0) return true;
        return false;
    }
    void tq_add(int rank, int type, int server) { tq[std::make_tuple(rank, type, server)]++; }
    void tq_dec(int rank, int type, int server) {
        auto it = tq.find(std::make_tuple(rank, type, server));
        if (it != tq.end() && --it->second <= 0) tq.erase(it);
    }
    // SS_RFRs a steal group leaves to its next round: their engine records (rfr_to_rank /
    // rfr_out) are cleared together by flush_rfr_cleared, one launch for all of them
    std::vector<int> rfr_cleared;
    int flush_rfr_cleared() {
        const int n = (int)rfr_cleared.size() / 2;
        if (!n) return 0;
        const int r = adlbq_rfr_done_batch(q, n, rfr_cleared.data());
        rfr_cleared.clear();
        return rc(r, "adlbq_rfr_done_batch");
    }
    void send_rfr(int donor, int rqseqno, const Parked &p) {
        // in a steal group the next round answers it, unless the donor holds targeted work for the rank;
        // the engine recorded the SS_RFR as outstanding (rfr_to_rank / rfr_out): clear that before the
        // next engine call, as the SS_RFR_RESP that never comes would (adlb.c:1877-1878), so a later
        // check_remote (a targeted Put for the rank landing elsewhere) does not skip the rank as busy
        if (grp && !tq_has(p.rank, donor)) {
            rfr_cleared.push_back(donor);
            rfr_cleared.push_back(p.rank);
            if (!want_sent) {  // ask the master for a round (once per round)
                want_sent = true;
                send(master, TAG_SRV_STEAL_WANT, nullptr, 0);
            }
            return;
        }
        rfr_sent++;
        int b[WIRE_RFR] = {rqseqno, p.rank};
        std::memcpy(b + 2, p.types, sizeof(p.types));
        send_ints(donor, TAG_SS_RFR, b, WIRE_RFR);
        rfr_out++;
    }
    void served(int rqseqno) {  // a parked Reserve got its answer (time_on_rq, adlb.c:1015-1021)
        auto it = parked.find(rqseqno);
        if (it == parked.end()) return;
        const int r = it->second.rank;
        if (r >= 0 && r < A && first_time_on_rq[r]) first_time_on_rq[r] = 0;
        else {
            time_on_rq += now() - it->second.t;
            n_rq_timed++;
        }
        parked.erase(it);
        row_events++;
    }
    // check_remote_work_for_queued_apps (adlb.c:3536-3579)
    int check_remote() {
        if (flush_rfr_cleared()) return -1;
        int cnt = 0;
        const int cap = (int)parked.size();
        if (!cap) return 0;
        crem.resize(3 * (size_t)cap);
        if (rc(adlbq_check_remote(q, cap, crem.data(), &cnt), "adlbq_check_remote")) return -1;
        for (int i = 0; i < cnt; i++) {
            auto it = parked.find(crem[3 * i]);
            if (it != parked.end()) send_rfr(crem[3 * i + 2], crem[3 * i], it->second);
        }
        return flush_rfr_cleared();
    }
    // answer every parked Reserve with code, FIFO order (adlb.c:1412-1442, 1639-1649)
    int drain_rq(int code) {
        if (parked.empty()) return 0;
        int count = 0;
        rqx.resize(18 * (parked.size() + 1));  // room for one more: an engine holding more is caught too
        if (rc(adlbq_rq_export(q, (int)parked.size() + 1, rqx.data(), &count), "adlbq_rq_export")) return -1;
        // the engine's rq and the host's parked map hold the same Reserves; a
        // disagreement would leave apps waiting forever: fail loudly instead
        if (count != (int)parked.size())
            return fail("drain_rq: the engine holds " + std::to_string(count) + " parked Reserves, the server " +
                        std::to_string(parked.size()));
        for (int i = 0; i < count; i++)
            if (!parked.count(rqx[18 * (size_t)i]))
                return fail("drain_rq: parked rqseqno " + std::to_string(rqx[18 * (size_t)i]) + " unknown to the server");
        std::vector<int> seqs((size_t)count), found((size_t)count);
        for (int i = 0; i < count; i++) {
            send_rc(rqx[18 * (size_t)i + 1], TAG_RESERVE_RESP, code);
            seqs[(size_t)i] = rqx[18 * (size_t)i];
        }
        if (count && rc(adlbq_rq_delete_batch(q, count, seqs.data(), found.data()), "adlbq_rq_delete_batch"))
            return -1;
        parked.clear();
        row_events++;
        return 0;
    }
};

extern "C" {

const char *adlbsrv_last_error(void) { return g_err.c_str(); }

int adlbsrv_create(adlbsrv **out, int ntypes, const int *user_types, int num_app_ranks, int num_servers,
                   int my_world_rank, double max_malloc, int device, adlbsrv_emit_fn emit, void *ctx) {
    if (!out || !emit || num_servers < 1 || my_world_rank < num_app_ranks ||
        my_world_rank >= num_app_ranks + num_servers)
        return fail("adlbsrv_create: bad argument");
    auto *s = new adlbsrv();
    s->T = ntypes;
    s->A = num_app_ranks;
    s->S = num_servers;
    s->me = my_world_rank;
    s->master = num_app_ranks;
    s->max_malloc = max_malloc;
    s->emit = emit;
    s->ctx = ctx;
    s->first_time_on_rq.assign((size_t)std::max(num_app_ranks, 1), 1);
    if (adlbq_create(&s->q, ntypes, user_types, num_app_ranks, num_servers, my_world_rank - num_app_ranks,
                     1 << 16, device)) {
        g_err = std::string("adlbq_create: ") + adlbq_last_error();
        delete s;
        return -1;
    }
    *out = s;
    return 0;
}

int adlbsrv_destroy(adlbsrv *s) {
    if (!s) return 0;
    if (s->grp) adlbq_steal_group_destroy(s->grp);
    if (s->q) adlbq_destroy(s->q);
    delete s;
    return 0;
}

static int put_reject(adlbsrv *s, int src, int len) {  // adlb.c:908-931 (nothing changed since the byte read)
    int rej = 0, hint = -1;
    if (s->rc(adlbq_put_check(s->q, len, s->max_malloc, &rej, &hint), "adlbq_put_check")) return -1;
    if (!rej) return fail("FA_PUT_HDR: memory check changed its answer");
    s->num_rejected++;
    int b[WIRE_IBUF] = {WIRE_PUT_REJECTED, hint, 1};
    s->send_ints(src, TAG_ACK_AND_RC, b, WIRE_IBUF);
    return 0;
}

int adlbsrv_put_hdr(adlbsrv *s, int src, const int *hdr, int *need_payload) {
    *need_payload = 0;
    if (s->nmw) {  // adlb.c:894-901
        s->send_rc(src, TAG_ACK_AND_RC, WIRE_NO_MORE_WORK);
        return 0;
    }
    const int len = hdr[4];
    if (!s->staged.empty()) {
        // curr_bytes_dmalloced after the staged Puts is at most hi (an rq match frees one parked
        // Reserve's node, adlb.c:1040, so it may be lower)
        const double hi = s->staged_base + s->staged_add;
        if (!(hi + len > s->max_malloc)) {  // accepted whatever the staged Puts match
            s->send_rc(src, TAG_ACK_AND_RC, WIRE_SUCCESS);
            *need_payload = 1;
            return 0;
        }
        if (adlbsrv_put_flush(s)) return -1;  // undecided, or a rejection: exact, from the appended queue
    }
    double curr = 0.0, hwm = 0.0;
    if (s->rc(adlbq_bytes(s->q, &curr, &hwm), "adlbq_bytes")) return -1;
    if (curr + len > s->max_malloc) return put_reject(s, src, len);  // adlb.c:908-931
    s->staged_base = curr;
    s->staged_add = 0.0;
    s->send_rc(src, TAG_ACK_AND_RC, WIRE_SUCCESS);  // adlb.c:960-961
    *need_payload = 1;
    return 0;
}

static void put_fields(const int *hdr, int *u) {
    const int v[ADLBQ_PUT_INTS] = {hdr[0], hdr[1], hdr[2], hdr[3], hdr[4], hdr[5], hdr[7], hdr[8], hdr[9]};
    std::memcpy(u, v, sizeof v);
}

// the append's replies (adlb.c:989-1049): the parked Reserve that gets the unit, then the final ack
static void put_done(adlbsrv *s, int src, const int *hdr, const int *u, const int *o, const char *buf, int len) {
    Unit &unit = s->units[o[0]];
    unit.buf.assign(buf, buf + (len > 0 ? len : 0));
    unit.t = now();
    std::memcpy(unit.fields, u, sizeof(int) * ADLBQ_PUT_INTS);
    unit.has_fields = true;
    s->activity++;
    if (o[1] >= 0) {
        int b[WIRE_IBUF] = {WIRE_SUCCESS, hdr[0], hdr[1], hdr[4], hdr[2], o[0], s->me, hdr[7], hdr[8], hdr[9]};
        s->send_ints(o[1], TAG_RESERVE_RESP, b, WIRE_IBUF);
        s->served(o[2]);
    }
    s->send_rc(src, TAG_ACK_AND_RC, WIRE_SUCCESS);
}

int adlbsrv_put_payload(adlbsrv *s, int src, const int *hdr, const void *buf, int len) {
    // wq_node_create + wq_append, then rq_find_rank_queued_for_type (adlb.c:963-988)
    if (!s->staged.empty() && adlbsrv_put_flush(s)) return -1;
    int u[ADLBQ_PUT_INTS], o[3];
    put_fields(hdr, u);
    if (s->rc(adlbq_put_batch(s->q, 1, u, o), "adlbq_put_batch")) return -1;
    put_done(s, src, hdr, u, o, (const char *)buf, len);
    return 0;
}

int adlbsrv_put_stage(adlbsrv *s, int src, const int *hdr, const void *buf, int len) {
    Staged st;
    st.src = src;
    put_fields(hdr, st.u);
    std::memcpy(st.hdr, hdr, sizeof st.hdr);
    st.buf.assign((const char *)buf, (const char *)buf + (len > 0 ? len : 0));
    s->staged.push_back(std::move(st));
    s->staged_add += (double)ADLBQ_BYTES_WQ + (double)(len > 0 ? len : 0);  // pmalloc + wq_node_create
    return 0;
}

int adlbsrv_put_staged(adlbsrv *s) { return (int)s->staged.size(); }

int adlbsrv_put_flush(adlbsrv *s) {
    const int n = (int)s->staged.size();
    if (!n) return 0;
    s->su.resize((size_t)n * ADLBQ_PUT_INTS);
    s->so.resize(3 * (size_t)n);
    for (int i = 0; i < n; i++) std::memcpy(&s->su[(size_t)i * ADLBQ_PUT_INTS], s->staged[(size_t)i].u, sizeof(int) * ADLBQ_PUT_INTS);
    std::vector<Staged> st;
    st.swap(s->staged);
    s->staged_add = 0.0;
    if (s->rc(adlbq_put_batch(s->q, n, s->su.data(), s->so.data()), "adlbq_put_batch")) return -1;
    for (int i = 0; i < n; i++) {
        const Staged &p = st[(size_t)i];
        put_done(s, p.src, p.hdr, &s->su[(size_t)i * ADLBQ_PUT_INTS], &s->so[3 * (size_t)i], p.buf.data(),
                 (int)p.buf.size());
    }
    return 0;
}

int adlbsrv_put_common_hdr(adlbsrv *s, int src, int common_len, int *need_payload) {
    *need_payload = 0;
    if (s->nmw) {
        s->send_rc(src, TAG_ACK_AND_RC, WIRE_NO_MORE_WORK);
        return 0;
    }
    int rej = 0, hint = -1;
    if (s->rc(adlbq_put_check(s->q, common_len, s->max_malloc, &rej, &hint), "adlbq_put_check")) return -1;
    if (rej) {  // adlb.c:1068-1093
        s->num_rejected++;
        int b[WIRE_IBUF] = {WIRE_PUT_REJECTED, hint, 1};
        s->send_ints(src, TAG_ACK_AND_RC, b, WIRE_IBUF);
        return 0;
    }
    s->send_rc(src, TAG_ACK_AND_RC, WIRE_SUCCESS);
    *need_payload = 1;
    return 0;
}

int adlbsrv_put_common_payload(adlbsrv *s, int src, const void *buf, int len) {
    // cq_node_create + cq_append (adlb.c:1127-1132); its bytes count like a put's
    Common &c = s->cq[s->next_cq];
    c.buf.assign((const char *)buf, (const char *)buf + (len > 0 ? len : 0));
    adlbq_bytes_adjust(s->q, (double)len);
    s->row_events++;  // nbytes_used of the row changed
    int b[WIRE_IBUF] = {WIRE_SUCCESS, s->next_cq};
    s->next_cq++;
    s->send_ints(src, TAG_ACK_AND_RC, b, WIRE_IBUF);
    return 0;
}

static void cq_maybe_free(adlbsrv *s, int cqseqno) {
    auto it = s->cq.find(cqseqno);
    if (it != s->cq.end() && it->second.refcnt == it->second.ngets) {  // cq_delete (adlb.c:1145, 1330)
        adlbq_bytes_adjust(s->q, -(double)it->second.buf.size());
        s->row_events++;
        s->cq.erase(it);
    }
}

int adlbsrv_batch_done(adlbsrv *s, int src, int cqseqno, int refcnt) {
    if (cqseqno > 0) {
        auto it = s->cq.find(cqseqno);
        if (it != s->cq.end()) {
            it->second.refcnt = refcnt;
            cq_maybe_free(s, cqseqno);
        }
    }
    s->send_rc(src, TAG_ACK_AND_RC, s->nmw ? WIRE_NO_MORE_WORK : WIRE_SUCCESS);
    return 0;
}

int adlbsrv_get_common(adlbsrv *s, int src, int cqseqno) {
    auto it = s->cq.find(cqseqno);
    if (it == s->cq.end()) return fail("FA_GET_COMMON: unknown common seqno " + std::to_string(cqseqno));
    s->send(src, TAG_GET_COMMON_RESP, it->second.buf.data(), (int)it->second.buf.size());
    it->second.ngets++;
    cq_maybe_free(s, cqseqno);
    return 0;
}

int adlbsrv_did_put_at_remote(adlbsrv *s, int type, int target, int server_rank) {
    if (s->rc(adlbq_tq_add(s->q, target, type, server_rank), "adlbq_tq_add")) return -1;
    s->tq_add(target, type, server_rank);
    return s->check_remote();  // adlb.c:1179
}

int adlbsrv_reserve_batch(adlbsrv *s, int n, const int *src, const int *bufs17) {
    s->num_reserves += n;
    if (s->nmw) {  // adlb.c:1192-1198
        for (int i = 0; i < n; i++) s->send_rc(src[i], TAG_RESERVE_RESP, WIRE_NO_MORE_WORK);
        return 0;
    }
    s->reqs.resize((size_t)n * ADLBQ_RESERVE_INTS);
    s->resp.resize((size_t)n * ADLBQ_RESP_INTS);
    for (int i = 0; i < n; i++) {
        int *r = s->reqs.data() + (size_t)i * ADLBQ_RESERVE_INTS;
        r[0] = src[i];
        std::memcpy(r + 1, bufs17 + (size_t)i * 17, sizeof(int) * 17);
    }
    if (s->rc(adlbq_reserve_batch(s->q, n, s->reqs.data(), s->resp.data()), "adlbq_reserve_batch")) return -1;
    const double t = now();
    for (int i = 0; i < n; i++) {
        int *r = s->resp.data() + (size_t)i * ADLBQ_RESP_INTS;
        if (r[0] == 1) {  // adlb.c:1207-1224
            int b[WIRE_IBUF];
            std::memcpy(b, r, sizeof(int) * 10);
            b[10] = b[11] = 0;
            s->send_ints(src[i], TAG_RESERVE_RESP, b, WIRE_IBUF);
            s->activity++;
        } else if (r[0] == -2) {  // adlb.c:1311-1316
            s->send_rc(src[i], TAG_RESERVE_RESP, WIRE_NO_CURR_WORK);
        } else {  // parked (adlb.c:1240-1309)
            Parked &p = s->parked[r[10]];
            p.rank = src[i];
            std::memcpy(p.types, s->reqs.data() + (size_t)i * ADLBQ_RESERVE_INTS + 2, sizeof(p.types));
            p.t = t;
            s->num_put_on_rq++;
            s->row_events++;
            if (r[11] >= 0) s->send_rfr(r[11], r[10], p);
        }
    }
    return s->flush_rfr_cleared();
}

int adlbsrv_get_batch(adlbsrv *s, int n, const int *src, const int *wqseqno) {
    if (s->nmw) {  // adlb.c:1340-1346
        for (int i = 0; i < n; i++) {
            double d[WIRE_IBUF] = {(double)WIRE_NO_MORE_WORK};
            s->send(src[i], TAG_ACK_AND_RC, d, (int)sizeof d);
        }
        return 0;
    }
    s->pairs.resize(2 * (size_t)n);
    s->out5.resize(5 * (size_t)n);
    for (int i = 0; i < n; i++) {
        s->pairs[2 * (size_t)i] = src[i];
        s->pairs[2 * (size_t)i + 1] = wqseqno[i];
    }
    if (s->rc(adlbq_get_reserved_batch(s->q, n, s->pairs.data(), s->out5.data()), "adlbq_get_reserved_batch"))
        return -1;
    const double t = now();
    int bad = 0;
    for (int i = 0; i < n; i++) {
        const int *o = s->out5.data() + 5 * (size_t)i;
        auto it = o[0] == 1 ? s->units.find(wqseqno[i]) : s->units.end();
        if (it == s->units.end()) {  // adlb.c:1349-1358
            double d[WIRE_IBUF] = {(double)WIRE_ERROR};
            s->send(src[i], TAG_ACK_AND_RC, d, (int)sizeof d);
            bad++;
            continue;
        }
        double d[WIRE_IBUF] = {(double)WIRE_SUCCESS, (double)o[1], t - it->second.t};
        s->send(src[i], TAG_ACK_AND_RC, d, (int)sizeof d);  // adlb.c:1360-1366
        s->send(src[i], TAG_GET_RESERVED_RESP, it->second.buf.data(), (int)it->second.buf.size());
        s->units.erase(it);
        s->activity++;
    }
    if (bad) return fail("FA_GET_RESERVED: " + std::to_string(bad) + " unit(s) not reserved for the rank");
    return 0;
}

int adlbsrv_info_num(adlbsrv *s, int src, int work_type) {
    int b[WIRE_IBUF] = {ADLBQ_LOWEST_PRIO, 0, 0, s->nmw ? WIRE_NO_MORE_WORK : 0};
    if (s->rc(adlbq_info_type(s->q, work_type, &b[0], &b[1], &b[2]), "adlbq_info_type")) return -1;
    s->send_ints(src, TAG_ACK_AND_RC, b, WIRE_IBUF);
    return 0;
}

int adlbsrv_no_more_work(adlbsrv *s) {
    const int fresh = !s->nmw;
    s->nmw = true;
    if (s->drain_rq(WIRE_NO_MORE_WORK)) return -1;
    return fresh;
}

int adlbsrv_exhausted(adlbsrv *s) { return s->drain_rq(WIRE_DONE_BY_EXHAUSTION); }

int adlbsrv_qmstat(adlbsrv *s, const int *qlen, const double *nbytes, const int *hi) {
    const int mine = s->me - s->master;
    for (int i = 0; i < s->S; i++)
        if (i != mine &&
            s->rc(adlbq_set_qmstat_row(s->q, i, qlen[i], nbytes[i], hi + (size_t)i * s->T), "adlbq_set_qmstat_row"))
            return -1;
    s->table_events++;
    return s->check_remote();  // adlb.c:1755
}

int adlbsrv_my_row(adlbsrv *s, int *qlen, double *nbytes, int *hi) {
    if (s->rc(adlbq_qmstat_row(s->q, qlen, hi), "adlbq_qmstat_row")) return -1;
    double hwm;
    return s->rc(adlbq_bytes(s->q, nbytes, &hwm), "adlbq_bytes");
}

int adlbsrv_rfr(adlbsrv *s, int src, const int *b) {
    // the donor side: wq_find_pre_targeted_hi_prio(for_rank) then wq_find_hi_prio, pin (adlb.c:1807-1827)
    int req[ADLBQ_RESERVE_INTS] = {b[1], 0};
    std::memcpy(req + 2, b + 2, sizeof(int) * WIRE_REQ);
    int r[ADLBQ_RESP_INTS];
    if (s->rc(adlbq_reserve_batch(s->q, 1, req, r), "adlbq_reserve_batch")) return -1;
    int o[WIRE_RFR] = {0};
    if (r[0] == 1) {  // adlb.c:1821-1846
        int prev_target = -1;
        if (s->rc(adlbq_unit_target(s->q, r[5], &prev_target), "adlbq_unit_target")) return -1;
        const int v[12] = {WIRE_SUCCESS, b[0], b[1], r[1], r[2], r[3], r[4], r[5], prev_target, r[7], r[8], r[9]};
        std::memcpy(o, v, sizeof v);
        s->activity++;
    } else {  // adlb.c:1848-1863
        s->row_events++;  // update_local_state after the miss (adlb.c:1863): the row goes out again
        o[0] = WIRE_NO_CURR_WORK;
        o[1] = b[0];
        o[2] = b[1];
        std::memcpy(o + 3, b + 2, sizeof(int) * WIRE_REQ);
    }
    s->send_ints(src, TAG_SS_RFR_RESP, o, WIRE_RFR);
    return 0;
}

int adlbsrv_rfr_resp(adlbsrv *s, int src, const int *b) {
    const int code = b[0], rqseqno = b[1], for_rank = b[2];
    if (s->rc(adlbq_rfr_done(s->q, src, for_rank), "adlbq_rfr_done")) return -1;  // adlb.c:1877-1878
    if (s->rfr_out > 0) s->rfr_out--;
    if (code == WIRE_SUCCESS) {
        int found = 0;
        if (s->rc(adlbq_rq_delete(s->q, rqseqno, &found), "adlbq_rq_delete")) return -1;
        if (found) {  // adlb.c:1884-1947
            auto it = s->parked.find(rqseqno);
            const int rank = it != s->parked.end() ? it->second.rank : for_rank;
            int r[WIRE_IBUF] = {WIRE_SUCCESS, b[3], b[4], b[5], b[6], b[7], src, b[9], b[10], b[11]};
            s->send_ints(rank, TAG_RESERVE_RESP, r, WIRE_IBUF);
            s->served(rqseqno);
            s->activity++;
            if (for_rank == b[8]) {
                if (s->rc(adlbq_tq_dec(s->q, for_rank, b[3], src), "adlbq_tq_dec")) return -1;
                s->tq_dec(for_rank, b[3], src);
            }
        } else {  // a Put answered it meanwhile: give the unit back (adlb.c:1949-1963)
            int u[WIRE_IBUF] = {for_rank, b[7], b[8]};
            s->send_ints(src, TAG_SS_UNRESERVE, u, WIRE_IBUF);
        }
        return s->check_remote();  // adlb.c:1964
    }
    // failure: patch the donor's row and tq, retry this Reserve, then everyone (adlb.c:1966-2047)
    if (s->rc(adlbq_rfr_failed(s->q, src, for_rank, b + 3), "adlbq_rfr_failed")) return -1;
    int found = 0, donor = -1;
    if (s->rc(adlbq_rfr_retry(s->q, rqseqno, &found, &donor), "adlbq_rfr_retry")) return -1;
    if (found && donor >= 0) {
        auto it = s->parked.find(rqseqno);
        if (it != s->parked.end()) s->send_rfr(donor, rqseqno, it->second);
    }
    return s->check_remote();
}

int adlbsrv_unreserve(adlbsrv *s, int src, const int *b) {
    (void)src;
    int found = 0;
    if (s->rc(adlbq_unreserve(s->q, b[0], b[1], b[2], &found), "adlbq_unreserve")) return -1;
    s->activity++;
    return 0;
}

// ---------------------------------------------------------------- push (adlb.c:509-556, 2109-2362)
static double threshold_to_start_push(const adlbsrv *s) { return 0.95 * s->max_malloc; }  // adlb.c:93

int adlbsrv_push_tick(adlbsrv *s) {
    if (s->push_out || s->S < 2) return 0;  // adlb.c:511
    // the condition only changes with queue or table events: skip the device read when none happened
    const long long stamp = s->activity + s->table_events;
    if (stamp == s->push_seen) return 0;
    double curr = 0, hwm = 0;
    if (s->rc(adlbq_bytes(s->q, &curr, &hwm), "adlbq_bytes")) return -1;
    if (!(curr > threshold_to_start_push(s))) {  // adlb.c:509
        s->push_seen = stamp;
        return 0;
    }
    int cand = -1, seq = -1;
    if (s->rc(adlbq_push_select(s->q, threshold_to_start_push(s), &cand, &seq), "adlbq_push_select")) return -1;
    if (cand < 0 || seq < 0) {  // no unpinned unit or no server below the threshold (adlb.c:513-529)
        s->push_seen = stamp;
        return 0;
    }
    // the unit's fields: its target from the engine, the rest kept from the Put
    auto it = s->units.find(seq);
    int tgt = -1;
    if (s->rc(adlbq_unit_target(s->q, seq, &tgt), "adlbq_unit_target")) return -1;
    int qa[ADLBQ_PUT_INTS];
    if (it == s->units.end() || !it->second.has_fields) return fail("push: no record of unit " + std::to_string(seq));
    std::memcpy(qa, it->second.fields, sizeof qa);
    double d[WIRE_IBUF] = {(double)qa[0], (double)qa[1], (double)qa[4], (double)qa[2], it->second.t, (double)tgt,
                           (double)qa[5], (double)seq, (double)qa[6], (double)qa[7], (double)qa[8]};
    s->send(cand, TAG_SS_PUSH_QUERY, d, (int)sizeof d);  // adlb.c:531-550
    s->push_out = true;
    return 1;
}

int adlbsrv_push_query(adlbsrv *s, int src, const double *d) {
    // the pushee (adlb.c:2113-2160): room for it below the threshold, or a decline
    double curr = 0, hwm = 0;
    if (s->rc(adlbq_bytes(s->q, &curr, &hwm), "adlbq_bytes")) return -1;
    const int len = (int)d[2];
    double r[WIRE_IBUF] = {-1.0, curr, d[7], 0.0};
    if (curr + len >= threshold_to_start_push(s)) {  // adlb.c:2122-2134
        r[3] = -1.0;  // (the reference sends the seqno it would have had; a decline never uses it)
        s->send(src, TAG_SS_PUSH_QUERY_RESP, r, (int)sizeof r);
        return 0;
    }
    Held h;
    h.type = (int)d[0];
    h.prio = (int)d[1];
    h.len = len;
    h.answer = (int)d[3];
    h.target = (int)d[5];
    h.home = (int)d[6];
    h.clen = (int)d[8];
    h.csrv = (int)d[9];
    h.cseq = (int)d[10];
    h.t = d[4];  // steady_clock seconds: one clock for every server process of a node
    const int u[ADLBQ_PUT_INTS] = {h.type, h.prio, h.answer, h.target, h.len, h.home, h.clen, h.csrv, h.cseq};
    int seq = -1;
    if (s->rc(adlbq_push_accept(s->q, u, &seq), "adlbq_push_accept")) return -1;
    r[0] = (double)s->me;
    r[3] = (double)seq;  // next_wqseqno (adlb.c:2139)
    s->send(src, TAG_SS_PUSH_QUERY_RESP, r, (int)sizeof r);
    s->held[seq] = h;
    s->activity++;
    return 0;
}

int adlbsrv_push_query_resp(adlbsrv *s, int src, const double *d) {
    // the pusher (adlb.c:2162-2225)
    const int to = (int)d[0];
    s->push_out = false;
    if (s->rc(adlbq_set_qmstat_nbytes(s->q, src - s->master, d[1]), "adlbq_set_qmstat_nbytes")) return -1;
    s->table_events++;  // the table changed: the loop-top check looks again
    if (to < 0) return 0;
    int o[10];
    if (s->rc(adlbq_push_take(s->q, (int)d[2], o), "adlbq_push_take")) return -1;
    int b[WIRE_IBUF] = {(int)d[3]};
    if (o[0] != 1) {  // a Reserve or a Get took it meanwhile (adlb.c:2182-2192)
        s->send_ints(to, TAG_SS_PUSH_DEL, b, WIRE_IBUF);
        return 0;
    }
    s->send_ints(to, TAG_SS_PUSH_HDR, b, WIRE_IBUF);  // adlb.c:2194-2207
    auto it = s->units.find((int)d[2]);
    if (it != s->units.end()) {
        s->send(to, TAG_SS_PUSH_WORK, it->second.buf.data(), (int)it->second.buf.size());
        s->units.erase(it);
    } else {
        s->send(to, TAG_SS_PUSH_WORK, nullptr, 0);
    }
    s->npushed_from++;
    return 0;
}

int adlbsrv_push_len(adlbsrv *s, int wqseqno) {
    auto it = s->held.find(wqseqno);
    return it == s->held.end() ? -1 : it->second.len;
}

int adlbsrv_push_hdr(adlbsrv *s, int src, const int *b, const void *payload, int len) {
    // the pushee (adlb.c:2228-2346)
    const int seq = b[0];
    auto hit = s->held.find(seq);
    if (hit == s->held.end()) return fail("SS_PUSH_HDR: invalid wqseqno " + std::to_string(seq));  // adlb.c:2233-2238
    const Held h = hit->second;
    s->held.erase(hit);
    int o[3];
    if (s->rc(adlbq_push_commit(s->q, seq, o), "adlbq_push_commit")) return -1;
    if (o[0] != 1) return fail("SS_PUSH_HDR: wqseqno " + std::to_string(seq) + " not held");
    Unit &unit = s->units[seq];
    unit.buf.assign((const char *)payload, (const char *)payload + (len > 0 ? len : 0));
    unit.t = h.t;  // ws->time_stamp = dbls_info_buf[4] (adlb.c:2150): the queued time keeps counting
    const int f[ADLBQ_PUT_INTS] = {h.type, h.prio, h.answer, h.target, h.len, h.home, h.clen, h.csrv, h.cseq};
    std::memcpy(unit.fields, f, sizeof f);
    unit.has_fields = true;
    s->npushed_to++;
    s->activity++;
    if (h.target >= 0) {  // adlb.c:2246-2272
        if (h.home == s->me) {
            if (s->rc(adlbq_tq_dec(s->q, h.target, h.type, src), "adlbq_tq_dec")) return -1;
            s->tq_dec(h.target, h.type, src);
        } else {
            int m[WIRE_IBUF] = {h.target, h.type, src, s->me};
            s->send_ints(h.home, TAG_SS_MOVING_TARGETED_WORK, m, WIRE_IBUF);
        }
    }
    if (o[1] >= 0) {  // a parked Reserve takes it (adlb.c:2287-2339)
        int r[WIRE_IBUF] = {WIRE_SUCCESS, h.type, h.prio, h.len, h.answer, seq, s->me, h.clen, h.csrv, h.cseq};
        s->send_ints(o[1], TAG_RESERVE_RESP, r, WIRE_IBUF);
        s->served(o[2]);
    }
    return 0;
}

int adlbsrv_push_del(adlbsrv *s, int src, const int *b) {
    (void)src;
    int found = 0;
    if (s->rc(adlbq_push_discard(s->q, b[0], &found), "adlbq_push_discard")) return -1;
    if (!found) return fail("SS_PUSH_DEL: invalid wqseqno " + std::to_string(b[0]));  // adlb.c:2354-2359
    s->held.erase(b[0]);
    s->activity++;
    return 0;
}

int adlbsrv_moving_targeted(adlbsrv *s, int src, const int *b) {
    // the home server's tq follows the unit (adlb.c:2075-2106)
    (void)src;
    if (s->rc(adlbq_tq_dec(s->q, b[0], b[1], b[2]), "adlbq_tq_dec")) return -1;
    s->tq_dec(b[0], b[1], b[2]);
    if (b[3] != s->me) {
        if (s->rc(adlbq_tq_add(s->q, b[0], b[1], b[3]), "adlbq_tq_add")) return -1;
        s->tq_add(b[0], b[1], b[3]);
    }
    return s->check_remote();
}

// ---------------------------------------------------------------- steal group
int adlbsrv_group_create(adlbsrv *s, int k, int rqcap) {
    if (s->grp) return 0;
    return s->rc(adlbq_steal_group_create(&s->grp, &s->q, 1, k, rqcap), "adlbq_steal_group_create");
}

long long adlbsrv_group_blob_ints(adlbsrv *s) { return s->grp ? adlbq_steal_group_blob_ints(s->grp) : -1; }

int adlbsrv_group_export(adlbsrv *s, int *blob) {
    if (!s->grp) return fail("adlbsrv_group_export: no steal group");
    return s->rc(adlbq_steal_group_export_host(s->grp, blob), "adlbq_steal_group_export_host");
}

int adlbsrv_group_export_device(adlbsrv *s, int *d_blob) {
    if (!s->grp) return fail("adlbsrv_group_export_device: no steal group");
    return s->rc(adlbq_steal_group_export(s->grp, d_blob), "adlbq_steal_group_export");
}

static int group_settle_common(adlbsrv *s, int *settled);

int adlbsrv_group_settle(adlbsrv *s, const int *all, int nproc, int *settled) {
    // the round's SS_RFR_RESP successes (adlb.c:1877-1948) for this server's
    // parked Reserves, and its donor side (1807-1827) for the others'
    if (!s->grp) return fail("adlbsrv_group_settle: no steal group");
    int nd = 0, won = 0;
    if (s->rc(adlbq_steal_group_settle_host(s->grp, all, nproc, &nd, &won), "adlbq_steal_group_settle_host"))
        return -1;
    return group_settle_common(s, settled);
}

int adlbsrv_group_settle_device(adlbsrv *s, const int *d_all, int nproc, int *settled) {
    // the blobs all-gathered in device memory (RCCL): the engine copies them to pinned memory once
    if (!s->grp) return fail("adlbsrv_group_settle_device: no steal group");
    int nd = 0, won = 0;
    if (s->rc(adlbq_steal_group_settle(s->grp, d_all, nproc, &nd, &won), "adlbq_steal_group_settle")) return -1;
    return group_settle_common(s, settled);
}

static int group_settle_common(adlbsrv *s, int *settled) {
    int cnt = 0;
    if (s->rc(adlbq_steal_group_responses(s->grp, 0, nullptr, &cnt), "adlbq_steal_group_responses")) return -1;
    s->grp_rows.resize(15 * (size_t)cnt);
    if (cnt && s->rc(adlbq_steal_group_responses(s->grp, cnt, s->grp_rows.data(), &cnt), "adlbq_steal_group_responses"))
        return -1;
    for (int i = 0; i < cnt; i++) {
        const int *r = s->grp_rows.data() + 15 * (size_t)i;
        auto it = s->parked.find(r[1]);
        if (it == s->parked.end() || it->second.rank != r[2])
            return fail("steal round: settled rqseqno " + std::to_string(r[1]) + " is not parked here");
        int b[WIRE_IBUF];
        std::memcpy(b, r + 3, sizeof(int) * 10);
        b[0] = WIRE_SUCCESS;
        b[10] = b[11] = 0;
        s->send_ints(r[2], TAG_RESERVE_RESP, b, WIRE_IBUF);
        s->served(r[1]);
        s->activity++;
    }
    int ng = 0;
    if (s->rc(adlbq_steal_group_grants(s->grp, 0, nullptr, &ng), "adlbq_steal_group_grants")) return -1;
    s->activity += ng;  // units this server pinned for other servers' apps
    if (ng) s->row_events++;
    int bad_g = 0, bad_d = 0;
    if (s->rc(adlbq_steal_group_check(s->grp, &bad_g, &bad_d), "adlbq_steal_group_check")) return -1;
    if (bad_g || bad_d)
        return fail("steal round: " + std::to_string(bad_g) + " grant(s) found their unit taken, " +
                    std::to_string(bad_d) + " settled Reserve(s) no longer parked");
    s->grp_rounds++;
    s->grp_settled += cnt;
    s->want_sent = false;
    if (settled) *settled = cnt;
    // Reserves the round could not reach (past rqcap, or behind an undecided one) wait for the next
    // round; those a tq donor can serve get their SS_RFR now (the export cleared every RFR record)
    return s->check_remote();
}

long long adlbsrv_group_stat(adlbsrv *s, int which) {
    switch (which) {
    case 0: return s->grp_rounds;
    case 1: return s->grp_settled;
    case 2: return s->rfr_sent;
    default: return -1;
    }
}

int adlbsrv_num_parked(adlbsrv *s) { return (int)s->parked.size(); }
long long adlbsrv_activity(adlbsrv *s) { return s->activity; }
long long adlbsrv_row_stamp(adlbsrv *s) { return s->activity + s->row_events; }  // both only grow
int adlbsrv_rfr_outstanding(adlbsrv *s) { return s->rfr_out; }
int adlbsrv_nmw(adlbsrv *s) { return s->nmw ? 1 : 0; }

int adlbsrv_info_get(adlbsrv *s, int key, double *val) {
    double curr = 0, hwm = 0;
    int wq = 0, wqmax = 0, rq = 0;
    switch (key) {
    case 1:  // ADLB_INFO_MALLOC_HWM
        if (s->rc(adlbq_bytes(s->q, &curr, &hwm), "adlbq_bytes")) return -1;
        *val = hwm;
        return 0;
    case 2:  // ADLB_INFO_AVG_TIME_ON_RQ
        *val = s->n_rq_timed ? s->time_on_rq / (double)s->n_rq_timed : 0.0;
        return 0;
    case 3:  // ADLB_INFO_NPUSHED_FROM_HERE
        *val = (double)s->npushed_from;
        return 0;
    case 4:  // ADLB_INFO_NPUSHED_TO_HERE
        *val = (double)s->npushed_to;
        return 0;
    case 6: case 7: case 8: case 9:  // qmstat-ring timings: no ring here
        *val = 0.0;
        return 0;
    case 5:  // ADLB_INFO_NREJECTED_PUTS
        *val = (double)s->num_rejected;
        return 0;
    case 10:  // ADLB_INFO_NUM_RESERVES
        *val = (double)s->num_reserves;
        return 0;
    case 11:  // ADLB_INFO_NUM_RESERVES_PUT_ON_RQ
        *val = (double)s->num_put_on_rq;
        return 0;
    case 12:  // ADLB_INFO_MAX_WQ_COUNT
        if (s->rc(adlbq_info(s->q, &wq, &wqmax, &rq), "adlbq_info")) return -1;
        *val = (double)wqmax;
        return 0;
    default:
        return fail("adlbsrv_info_get: unknown key");
    }
}

}  // extern "C"
