import heapq, numpy as np, sys
rng=np.random.default_rng(0)
n, m, G = 4096, 2048, 8
S=63
cost = np.exp(rng.normal(np.log(6.5e6), 0.2, n)); cost = np.minimum(cost, 1.25e7)
pred = cost*np.exp(rng.normal(0,0.08,n))  # predicted (prev step) cost, corr ~0.92
def run(margin=0.25, yields=1, every=8, xcd=True, cont_pick='fifo', handoff=5e3*2.3):
    order = np.argsort(-pred)
    fresh = list(order)[::-1]   # pop from end = heaviest first
    done_sub = np.zeros(n, int); ny = np.zeros(n, int)
    queues = [[] for _ in range(G)]  # entries (rem_pred, env)
    home = -np.ones(n, int)
    t_free = [(0.0, w) for w in range(m)]
    heapq.heapify(t_free)
    busy = 0.0; end = 0.0
    per = cost/S
    while t_free:
        t, w = heapq.heappop(t_free)
        g = w % G if xcd else 0
        q = queues[g]
        # pick
        nextc = pred[fresh[-1]] if fresh else -1
        env = None
        if q:
            if cont_pick == 'fifo': cand = 0
            else: cand = max(range(len(q)), key=lambda i: q[i][0])
            if (not fresh) or q[cand][0] >= nextc:
                env = q.pop(cand)[1]
        if env is None and fresh:
            env = fresh.pop(); home[env] = g
        if env is None:
            # idle: wake when something may be queued -> approximate: retry later
            if any(queues) or fresh or (done_sub < S).any():
                heapq.heappush(t_free, (t + 2e4, w)); continue
            continue
        if env is not None and home[env] != g and xcd: raise Exception
        # run until yield or end
        k = S - done_sub[env]; tt = t + (handoff if done_sub[env] > 0 else 0)
        i = 0
        while i < k:
            if ny[env] < yields and i > 0 and i % every == 0 and fresh:
                # check at time tt + i*per: fresh state at that time (approx: current)
                left = pred[env]*(S - done_sub[env] - i)/S
                if left*(1+margin) < pred[fresh[-1]]: break
            i += 1
        run_t = i*per[env]
        done_sub[env] += i
        tt += run_t; busy += tt - t
        if done_sub[env] < S:
            ny[env] += 1
            queues[home[env] if xcd else 0].append((pred[env]*(S-done_sub[env])/S, env))
        end = max(end, tt)
        heapq.heappush(t_free, (tt, w))
    return end, busy/(m*end), cost.sum()/m
legacy_sorted = None
for args in [dict(yields=0), dict(margin=0.25), dict(margin=0.5), dict(margin=0.5, cont_pick='lrpt'), dict(margin=0.5, xcd=False), dict(margin=0.5,yields=3, cont_pick='lrpt', xcd=False), dict(margin=0.25,yields=8, cont_pick='lrpt', xcd=False, every=4)]:
    e,b,ideal = run(**args)
    print(args, 'span %.3e busy %.3f ideal %.3e ratio %.3f'%(e,b,ideal,e/ideal))
print('---')
for args in [dict(margin=0.5, yields=3, cont_pick='lrpt'), dict(margin=0.5, yields=3, cont_pick='fifo'), dict(margin=0.5, yields=2, cont_pick='lrpt'), dict(margin=1.0, yields=3, cont_pick='lrpt'), dict(margin=0.5, yields=3, cont_pick='lrpt', every=4), dict(margin=0.5, yields=6, cont_pick='lrpt', every=4), dict(margin=0.5, yields=3, cont_pick='lrpt', handoff=2e4*2.3)]:
    e,b,ideal = run(**args)
    print(args, 'span %.3e busy %.3f ideal %.3e ratio %.3f'%(e,b,ideal,e/ideal))
