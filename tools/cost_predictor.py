"""Developer study: which dispatch-cost predictor orders the C3 rollout launch best.

Reads tools/c3_cost_dump.py's per-env per-env-step clocks (T steps), cuts them into jobs of
R env-steps (one gm_rollout launch = one job per env), and for each launch k >= 1 replays
the chunked queue's policy (tools/sim_dispatch.py's model: envs started heaviest-predicted
first on m wave slots in G XCD groups, a running env yielding every `every` substeps to an
unstarted or yielded env with clearly more predicted work left) with the job's true cost
and a predictor built from what the kernel knows when launch k starts.  Prints each
predictor's makespan over the ideal (total work / slots).
usage: python tools/cost_predictor.py <c3_costs.npz> [R] [slots]"""
import heapq
import sys

import numpy as np


def run(cost, pred, m, G=8, S=630, margin=0.5, cmargin=0.5, every=16, yields=20, handoff=2e4):
    n = len(cost)
    fresh = list(np.argsort(-pred, kind="stable"))[::-1]      # pop() = heaviest unstarted
    done_sub = np.zeros(n, int)
    ny = np.zeros(n, int)
    queues = [[] for _ in range(G)]
    home = -np.ones(n, int)
    free = [(0.0, w) for w in range(m)]
    heapq.heapify(free)
    end = 0.0
    per = cost / S
    while free:
        t, w = heapq.heappop(free)
        g = w % G
        q = queues[g]
        env = None
        if q:
            c = max(range(len(q)), key=lambda i: q[i][0])
            if not fresh or q[c][0] >= pred[fresh[-1]]:
                env = q.pop(c)[1]
        if env is None and fresh:
            env = fresh.pop()
            home[env] = g
        if env is None:
            if any(queues) or fresh or (done_sub < S).any():
                heapq.heappush(free, (t + 2e4, w))
            continue
        k = S - done_sub[env]
        tt = t + (handoff if done_sub[env] > 0 else 0.0)
        i = 0
        while i < k:
            if ny[env] < yields and i > 0 and i % every == 0:
                left = pred[env] * (S - done_sub[env] - i) / S
                if fresh and left * (1 + margin) < pred[fresh[-1]]:
                    break
                if q and left * (1 + cmargin) < max(x[0] for x in q):
                    break
            i += 1
        tt += i * per[env]
        done_sub[env] += i
        if done_sub[env] < S:
            ny[env] += 1
            queues[home[env]].append((pred[env] * (S - done_sub[env]) / S, env))
        end = max(end, tt)
        heapq.heappush(free, (tt, w))
    return end / (cost.sum() / m)


def main(path, R=10, m=2048):
    d = np.load(path)
    cyc, nefc, newton, mpr = d["cyc"], d["nefc"], d["newton"], d["mpr"]
    T, n = cyc.shape
    R, m = int(R), int(m)
    K = T // R
    jobs = np.stack([cyc[k * R:(k + 1) * R].sum(0) for k in range(K)])
    preds = {
        "previous job (clocks)": lambda k: jobs[k - 1],
        "previous job (work model)": lambda k: (14000 * 64 * R + 19 * 64 * nefc[(k - 1) * R:k * R].sum(0)
                                               + 188 * 64 * mpr[(k - 1) * R:k * R].sum(0) + 940 * 64 * newton[(k - 1) * R:k * R].sum(0)),
        "kernel blend (clocks/2 + model/2)": lambda k: 0.5 * jobs[k - 1] + 0.5 * (
            14000 * 64 * R + 19 * 64 * nefc[(k - 1) * R:k * R].sum(0) + 188 * 64 * mpr[(k - 1) * R:k * R].sum(0)
            + 940 * 64 * newton[(k - 1) * R:k * R].sum(0)),
        "last env-step x R": lambda k: cyc[k * R - 1] * R,
        "last 3 env-steps x R/3": lambda k: cyc[k * R - 3:k * R].sum(0) * R / 3,
        "max(previous job, last step x R)": lambda k: np.maximum(jobs[k - 1], cyc[k * R - 1] * R),
        "0.5 previous job + 0.5 last step x R": lambda k: 0.5 * jobs[k - 1] + 0.5 * cyc[k * R - 1] * R,
        "oracle (true cost)": lambda k: jobs[k],
        "none (env order)": lambda k: -np.arange(n, dtype=np.float64),
    }
    print(f"{n} envs, {T} env-steps -> {K} launches of R = {R}; job cost max/mean "
          + ", ".join(f"{jobs[k].max() / jobs[k].mean():.2f}" for k in range(K)))
    for name, f in preds.items():
        r = [run(jobs[k], f(k).astype(np.float64), m, S=63 * R) for k in range(1, K)]
        cc = [np.corrcoef(f(k), jobs[k])[0, 1] for k in range(1, K)]
        print(f"  {name:40s} makespan/ideal " + " ".join(f"{x:.3f}" for x in r) + f"   corr " + " ".join(f"{x:.2f}" for x in cc))


if __name__ == "__main__":
    main(*sys.argv[1:])
