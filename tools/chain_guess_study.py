"""Chain guess study: on a synthetic config-2 batch
(random type interleaving of the candidates, 70/20/10 single/pair/wildcard
requests), how many requests a replay started from a guessed state needs to
coalesce with the true sequential state: the level guess vs. a water-filling
guess and guesses corrected by recent single-type imbalance.  CPU only:
`python tools/chain_guess_study.py [seed]`."""
import numpy as np, sys
rng = np.random.default_rng(int(sys.argv[1]) if len(sys.argv) > 1 else 1)
T, R = 4, 65536
G = 100000
gt = rng.integers(0, T, size=G)                      # type of the candidate at global rank g
lists = [np.nonzero(gt == t)[0] for t in range(T)]  # global ranks per type (ascending)
u = rng.random(R)
masks = np.zeros(R, np.int64)
single = u < 0.7; pair = (u >= 0.7) & (u < 0.9); wild = u >= 0.9
a = rng.integers(0, T, R); b = (a + rng.integers(1, T, R)) % T
masks[single] = 1 << a[single]
masks[pair] = (1 << a[pair]) | (1 << b[pair])
masks[wild] = (1 << T) - 1
def step(pos, m):
    best, bt = None, -1
    for t in range(T):
        if (m >> t) & 1 and pos[t] < len(lists[t]):
            r = lists[t][pos[t]]
            if best is None or r < best: best, bt = r, t
    if bt >= 0: pos[bt] += 1
# true trajectory
S = np.zeros((R + 1, T), np.int64); pos = [0] * T
for j in range(R):
    S[j] = pos; step(pos, masks[j])
S[R] = pos
def level(J):
    return [int(np.searchsorted(lists[t], J)) for t in range(T)]
single_cnt = np.zeros((R + 1, T), np.int64)
for t in range(T):
    single_cnt[1:, t] = np.cumsum(masks == (1 << t))
def water(J, j):
    s = single_cnt[j]
    lo, hi = 0, G
    while lo < hi:  # smallest lam with sum max(s, L(lam)) >= J
        mid = (lo + hi) // 2
        v = sum(max(int(s[t]), int(np.searchsorted(lists[t], mid))) for t in range(T))
        if v >= J: hi = mid
        else: lo = mid + 1
    return [max(int(s[t]), int(np.searchsorted(lists[t], lo))) for t in range(T)]
def coal(g, j0, limit=4096):
    pos = list(g)
    for k in range(limit):
        if all(pos[t] == S[j0 + k][t] for t in range(T)): return k
        if j0 + k >= R: return limit
        step(pos, masks[j0 + k])
    return limit
res = {'level': [], 'water': []}
for js in range(1024, R - 1024, 256):
    J = int(S[js].sum())
    res['level'].append(coal(level(J), js))
    res['water'].append(coal(water(J, js), js))
for k, v in res.items():
    v = np.array(v)
    print(k, "median", np.median(v), "p90", np.percentile(v, 90), "p97", np.percentile(v, 97), "p99", np.percentile(v, 99), "max", v.max(), "frac<=256", (v <= 256).mean(), "frac<=128", (v <= 128).mean())
devs = []
for js in range(1024, R - 1024, 256):
    J = int(S[js].sum()); L = level(J)
    devs.append([int(S[js][t]) - L[t] for t in range(T)])
devs = np.array(devs)
print("dev mean", devs.mean(0), "abs mean", np.abs(devs).mean(), "max abs", np.abs(devs).max())
print(devs[:10])
# guess: level at J, corrected by single-type imbalance over the last W requests
for W in (128, 256, 512):
    out = []
    for js in range(1024, R - 1024, 256):
        J = int(S[js].sum()); L = np.array(level(J))
        s = single_cnt[js] - single_cnt[js - W]
        c = s - s.mean()
        g = np.maximum(0, L + np.round(c * 0.5).astype(int))
        g = g + (J - g.sum()) // T
        out.append(coal(list(g), js))
    out = np.array(out)
    print("corr W", W, "median", np.median(out), "p97", np.percentile(out, 97), "max", out.max())
