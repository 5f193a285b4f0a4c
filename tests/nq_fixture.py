"""Replay of a recorded reference server event stream (oracle/gen_nq.py
fixtures) through the repo's server core, and the reply comparison.

Replies are compared on the fields the reference defines; words the
reference leaves uninitialised on the wire (the tails of int[12] acks, the
queued time of a Get) are not compared.
"""
from __future__ import annotations

import numpy as np

KIND = {1: "put", 2: "reserve", 3: "get", 4: "info", 5: "nmw", 6: "ss_nmw", 7: "qmstat", 8: "rfr",
        9: "rfr_resp", 10: "unreserve", 11: "common_hdr", 12: "batch_done", 13: "get_common",
        14: "did_put_at_remote", 15: "exhausted"}
T_RESERVE_RESP, T_GET_RESP, T_ACK, T_RFR, T_RFR_RESP, T_UNRESERVE, T_GET_COMMON_RESP = (
    1008, 1010, 1020, 1018, 1019, 1028, 1039)
PUT_REJECTED = -999999996


class Fixture:
    def __init__(self, path):
        z = np.load(path)
        self.meta = z["meta"]
        self.types = z["types"]
        self.T, self.A, self.S, self.me, self.max_malloc = (int(x) for x in self.meta)
        eb, xb = z["ev_blob"].tobytes(), z["ex_blob"].tobytes()
        self.events = [(KIND[int(k)], int(s), eb[int(o):int(o) + int(n)])
                       for k, s, o, n in zip(z["ev_kind"], z["ev_src"], z["ev_off"], z["ev_len"])]
        self.replies = [(int(e), int(d), int(t), xb[int(o):int(o) + int(n)])
                        for e, d, t, o, n in zip(z["ex_ev"], z["ex_dest"], z["ex_tag"], z["ex_off"], z["ex_len"])]

    def expected(self):
        """[(kind of the causing event, dest, tag, bytes)] in sending order"""
        return [(self.events[e][0], d, t, b) for e, d, t, b in self.replies]

    def qmstat_table(self, blob):
        """The reference's packed table (adlb.c:3178-3198): per server hi[T] int, qlen int, nbytes double."""
        qlen, nbytes, hi = [], [], []
        row = 4 * self.T + 4 + 8
        for i in range(self.S):
            r = blob[i * row:(i + 1) * row]
            hi.extend(np.frombuffer(r[:4 * self.T], np.int32).tolist())
            qlen.append(int(np.frombuffer(r[4 * self.T:4 * self.T + 4], np.int32)[0]))
            nbytes.append(float(np.frombuffer(r[4 * self.T + 4:], np.float64)[0]))
        return qlen, nbytes, hi


def ints(b, n=None):
    v = np.frombuffer(b[: len(b) // 4 * 4], np.int32)
    return v if n is None else v[:n]


def normalise(kind, dest, tag, b):
    """The defined content of one reply."""
    if tag == T_RESERVE_RESP:
        v = ints(b)
        return (dest, tag, tuple(v[:10]) if v[0] == 1 else (int(v[0]),))
    if tag == T_ACK:
        if kind == "get":  # doubles {rc, len, queued time}
            d = np.frombuffer(b, np.float64)
            return (dest, tag, (float(d[0]), float(d[1])) if d[0] == 1 else (float(d[0]),))
        v = ints(b)
        if kind == "info":
            return (dest, tag, tuple(v[:4]))
        if v[0] == PUT_REJECTED:
            return (dest, tag, tuple(v[:3]))
        if kind == "common_hdr" and len(v) > 1 and v[0] == 1:
            return (dest, tag, (int(v[0]),))
        return (dest, tag, (int(v[0]),))
    if tag == T_RFR:
        return (dest, tag, tuple(ints(b, 18)))
    if tag == T_RFR_RESP:
        v = ints(b)
        return (dest, tag, tuple(v[:12]) if v[0] == 1 else tuple(v[:19]))
    if tag == T_UNRESERVE:
        return (dest, tag, tuple(ints(b, 3)))
    return (dest, tag, bytes(b))  # payloads


def replay(core, fx: Fixture, batch: bool = True, put_batch: bool = False):
    """Feed the fixture's events to a Core; returns [(kind, dest, tag, bytes)].
    put_batch: runs of Puts go through Core.put_run as libadlb.so drains them
    (replies then differ in order across destinations only: compare_per_dest)."""
    out = []
    ev = fx.events
    i = 0
    while i < len(ev):
        kind, src, b = ev[i]
        if kind in ("reserve", "get"):
            j = i + 1
            if batch:
                while j < len(ev) and ev[j][0] == kind:
                    j += 1
            srcs = [ev[k][1] for k in range(i, j)]
            if kind == "reserve":
                r = core.reserve_batch(srcs, np.stack([ints(ev[k][2], 17) for k in range(i, j)]))
            else:
                r = core.get_batch(srcs, [int(ints(ev[k][2])[0]) for k in range(i, j)])
            out.extend((kind, d, t, x) for d, t, x in r)
            i = j
            continue
        if kind == "put" and put_batch:
            j = i + 1
            while j < len(ev) and ev[j][0] == "put":
                j += 1
            r = core.put_run([(ev[k][1], ints(ev[k][2][:48]), ev[k][2][48:]) for k in range(i, j)])
            out.extend((kind, d, t, x) for d, t, x in r)
            i = j
            continue
        if kind == "put":
            r = core.put(src, ints(b[:48]), b[48:])
        elif kind == "common_hdr":
            r = core.put_common(src, int(ints(b[:48])[0]), b[48:])
        elif kind == "info":
            r = core.info_num(src, int(ints(b)[0]))
        elif kind in ("nmw", "ss_nmw"):
            r = core.no_more_work()
        elif kind == "exhausted":
            r = core.exhausted()
        elif kind == "qmstat":
            r = core.qmstat(*fx.qmstat_table(b))
        elif kind == "rfr":
            r = core.rfr(src, ints(b, 28))
        elif kind == "rfr_resp":
            r = core.rfr_resp(src, ints(b, 28))
        elif kind == "unreserve":
            r = core.unreserve(src, ints(b, 12))
        elif kind == "batch_done":
            v = ints(b)
            r = core.batch_done(src, int(v[0]), int(v[1]))
        elif kind == "get_common":
            r = core.get_common(src, int(ints(b)[0]))
        elif kind == "did_put_at_remote":
            v = ints(b)
            r = core.did_put_at_remote(int(v[0]), int(v[1]), int(v[2]))
        else:
            raise ValueError(kind)
        out.extend((kind, d, t, x) for d, t, x in r)
        i += 1
    return out


def compare(got, exp):
    """First mismatch as a message, or None."""
    g = [normalise(*x) for x in got]
    e = [normalise(*x) for x in exp]
    for k, (a, b) in enumerate(zip(g, e)):
        if a != b:
            return f"reply {k}: got {a} expected {b} (caused by {exp[k][0]})"
    if len(g) != len(e):
        return f"{len(g)} replies, expected {len(e)}"
    return None


def compare_per_dest(got, exp):
    """First mismatch of the reply sequence to some destination, or None: a
    batched run of Puts reorders replies across destinations only (MPI orders
    messages per sender-receiver pair)."""
    def by_dest(x):
        d = {}
        for r in x:
            n = normalise(*r)
            d.setdefault(n[0], []).append(n)
        return d
    g, e = by_dest(got), by_dest(exp)
    if set(g) != set(e):
        return f"destinations differ: got {sorted(g)} expected {sorted(e)}"
    for dest in sorted(e):
        for k, (a, b) in enumerate(zip(g[dest], e[dest])):
            if a != b:
                return f"dest {dest} reply {k}: got {a} expected {b}"
        if len(g[dest]) != len(e[dest]):
            return f"dest {dest}: {len(g[dest])} replies, expected {len(e[dest])}"
    return None
