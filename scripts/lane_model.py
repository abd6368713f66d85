"""Toy queueing models behind DESIGN.md §2 "Experiments" (N1, active-ray compaction).

Synthetic query lengths in traversal iterations (geometric with mean 6, plus a 30 % tail of up to 5
more); a traversal iteration costs 1, a shading phase S; a wave shades once W of its lanes wait.
- pool_model: 4 waves of 64 lanes, one path per lane, with and without pooling busy queries across
  waves at phase boundaries (move costs charged).
- paths_model: one wave of 64 lanes holding P >= 64 paths (queries wait for a free lane).
Printed: cost per query (lower is better) and lane utilisation. Output: profiles/r03_lane_model.txt.
"""
import numpy as np

rng = np.random.default_rng(1)
def qlen():
    # query length in traversal iterations: geometric-ish, mean ~6, heavy tail
    return 1 + rng.geometric(1/6.0) - 1 + (rng.random() < 0.3) * rng.integers(0, 6)

def pool_model(pool, W=56, S=12.0, waves=4, T=200000, move_cost=0.15, result_cost=0.05):
    # each wave: lanes rem[] (remaining iterations of the query the lane traverses; 0 = none),
    # own_done[] (own path's result ready), own_inflight (own query somewhere)
    rem = [np.zeros(64, int) for _ in range(waves)]
    owner = [np.full(64, -1) for _ in range(waves)]
    ready = [np.zeros(64, bool) for _ in range(waves)]
    inflight = [np.zeros(64, bool) for _ in range(waves)]
    for w in range(waves):
        for l in range(64):
            rem[w][l] = qlen(); owner[w][l] = w * 64 + l; inflight[w][l] = True
    poolq = []
    busy_until = [0.0] * waves
    t = [0.0] * waves
    issue = 0.0; lane_work = 0; queries = 0; iters = 0
    shading_cost = 0.0
    while queries < T:
        w = int(np.argmin(t))
        r, o = rem[w], owner[w]
        nready = ready[w].sum()
        nbusy = (r > 0).sum()
        if pool and len(poolq) and (r == 0).any():
            idle = np.where(r == 0)[0]
            k = min(len(idle), len(poolq))
            for i in idle[:k]:
                rr, oo = poolq.pop()
                r[i] = rr; o[i] = oo
            t[w] += move_cost * (k > 0)
            nbusy = (r > 0).sum()
        if nready >= min(W, nready + inflight[w].sum() - 0) and nready > 0 or (nbusy == 0 and nready > 0 and (not pool or True)):
            # gate: shade ready lanes
            if pool:
                busy = np.where(r > 0)[0]
                for i in busy:
                    poolq.append((r[i], o[i])); r[i] = 0; o[i] = -1
                t[w] += move_cost * (len(busy) > 0)
            n = ready[w].sum()
            t[w] += S
            shading_cost += S
            # shaded lanes issue new queries into own lanes if free else pool
            for l in np.where(ready[w])[0]:
                ready[w][l] = False; inflight[w][l] = True
                q = qlen()
                if r[l] == 0:
                    r[l] = q; o[l] = w * 64 + l
                else:
                    poolq.append((q, w * 64 + l))
            continue
        if nbusy == 0:
            t[w] += 1.0  # spin
            continue
        # one traversal iteration
        t[w] += 1.0; iters += 1
        act = r > 0
        lane_work += act.sum()
        r[act] -= 1
        fin = np.where(act & (r == 0))[0]
        for i in fin:
            ow = o[i] // 64; ol = o[i] % 64
            ready[ow][ol] = True; inflight[ow][ol] = False; o[i] = -1
            queries += 1
        if pool and len(fin):
            t[w] += result_cost
    total = max(t) * waves
    return total / queries, lane_work / (64 * iters), shading_cost / total

def pool_table():
    for W in (40, 48, 56, 60):
      for S in (8.0, 12.0):
        a = pool_model(False, W=W, S=S)
        b = pool_model(True, W=W, S=S)
        print(f"W={W} S={S}: no pool cost/query {a[0]:.3f} lanes {a[1]:.2f} shade {a[2]:.2f} | pool {b[0]:.3f} lanes {b[1]:.2f} shade {b[2]:.2f}  gain {a[0]/b[0]:.3f}")


def paths_model(P, W, S=10.0, T=100000, park_cost=0.0):
    # one wave, 64 lanes, P paths; queue of pending queries; shading batches of up to 64 ready paths
    rem = np.zeros(64, int)
    pending = [qlen() for _ in range(P)]
    ready = 0
    t = 0.0; lw = 0; it = 0; q = 0
    while q < T:
        idle = np.where(rem == 0)[0]
        k = min(len(idle), len(pending))
        for i in idle[:k]:
            rem[i] = pending.pop()
        if k: t += park_cost
        nb = (rem > 0).sum()
        if ready >= W or (nb == 0 and ready > 0):
            n = min(ready, 64)
            t += S * 1.0
            ready -= n
            pending.extend(qlen() for _ in range(n))
            continue
        t += 1; it += 1
        act = rem > 0
        lw += act.sum()
        rem[act] -= 1
        f = int((act & (rem == 0)).sum())
        ready += f; q += f
    return t / q, lw / (64 * it)

def paths_table():
  for S in (6.0, 10.0):
    print("S", S)
    for P, Ws in ((64, (40, 48, 56)), (96, (48, 56, 64)), (128, (56, 64))):
        for W in Ws:
            c, l = paths_model(P, W, S)
            print(f"  paths={P} W={W}: cost/query {c:.3f} lanes {l:.2f}")

if __name__ == "__main__":
    print("pooling across 4 waves (one path per lane)")
    pool_table()
    print("more paths than lanes (one wave)")
    paths_table()
