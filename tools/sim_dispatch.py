"""Developer model of the chunked env-step's dispatch (gm_kernels.hip chunked_env_steps):
list scheduling of n env-steps on m resident wave slots in G XCD groups, envs started in
descending predicted cost, a running env yielding every `every` substeps when the next
unstarted env (margin) or the best yielded env of its group (cmargin) has clearly more
work left, yielded envs resumed longest-work-left first.  Costs are lognormal around the
C3 workload's env-step cost (tools/tail_bench.py: mean 6.7e6 clocks, p90 8.5e6); the
prediction (last env-step's cost) is correlated ~0.92 with the true cost.  Prints each
policy's makespan over the ideal (total work / slots) and the wave-busy fraction.
usage: python tools/sim_dispatch.py"""
import heapq

import numpy as np

rng = np.random.default_rng(0)
n, m, G, S = 4096, 2048, 8, 63
cost = np.minimum(np.exp(rng.normal(np.log(6.5e6), 0.2, n)), 1.25e7)
pred = cost * np.exp(rng.normal(0, 0.08, n))


def run(margin=1.0, yields=6, every=8, cmargin=None, handoff=1e4, preempt=True):
    fresh = list(np.argsort(-pred))[::-1]      # pop() = heaviest unstarted
    done_sub = np.zeros(n, int)
    ny = np.zeros(n, int)
    queues = [[] for _ in range(G)]
    home = -np.ones(n, int)
    free = [(0.0, w) for w in range(m)]
    heapq.heapify(free)
    busy = end = 0.0
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
            if preempt and ny[env] < yields and i > 0 and i % every == 0:
                left = pred[env] * (S - done_sub[env] - i) / S
                if fresh and left * (1 + margin) < pred[fresh[-1]]:
                    break
                if cmargin is not None and q and left * (1 + cmargin) < max(x[0] for x in q):
                    break
            i += 1
        tt += i * per[env]
        done_sub[env] += i
        busy += tt - t
        if done_sub[env] < S:
            ny[env] += 1
            queues[home[env]].append((pred[env] * (S - done_sub[env]) / S, env))
        end = max(end, tt)
        heapq.heappush(free, (tt, w))
    return end / (cost.sum() / m), busy / (m * end)


if __name__ == "__main__":
    for a in [dict(preempt=False), dict(margin=0.25, yields=1), dict(margin=0.5, yields=1), dict(),
              dict(cmargin=1.0), dict(cmargin=0.5), dict(margin=2.0, cmargin=1.0, yields=10)]:
        print(a, "makespan / ideal %.3f  busy %.3f" % run(**a))
