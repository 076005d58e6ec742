"""The grounding launch's tail, simulated on the CPU from the C oracle's
per-query work (F, T, P) of the FB15k-237 split: 512 persistent workgroups
dequeue queries in a given order (greedy, earliest-free first); per-query
cost = a fixed 20 k-cycle part + the rest in proportion to 12 F + 12 T + 8 P,
calibrated to the measured 161 k cycles per query (tools/profile_phases.py).
Prints the makespan and tail for row order and heaviest-first orders.
Usage (this container): python tools/tail_sim.py"""
import sys, time, heapq
import numpy as np
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
import bench
from oracle import ground_c
graph, test_set, model, rows = bench.build_workload("bias")
cg = ground_c.CGraph(graph.entity_size, graph.relation_size, np.asarray(graph._train, dtype=np.int32))
cr = ground_c.CRules(model.rules, graph.relation_size)
o = ground_c.Oracle(cg, model.rules, graph.relation_size)
h = np.ascontiguousarray(rows[:, 0]); r = np.ascontiguousarray(rows[:, 1])
t = time.time()
d, c, w = o.digests(h, r, threads=8, work=True)
print("oracle %.1f s" % (time.time() - t))
F, T, P = w[:, 0].astype(float), w[:, 1].astype(float), w[:, 2].astype(float)
# cost model: per query a fixed latency part + work part (cycles); calibrate: total 161k cycles/query avg
base = 20000.0
cost = base + (12 * F + 12 * T + 8 * P) / (12 * F + 12 * T + 8 * P).mean() * (161000 - base)
np.save('/tmp/fb_query_cost.npy', cost)
def sim(order, workers=512):
    heap = [0.0] * workers
    for q in order:
        t0 = heapq.heappop(heap); heapq.heappush(heap, t0 + cost[q])
    return max(heap), sum(heap) / workers
for name, order in (("row order", np.arange(len(cost))), ("cost descending", np.argsort(-cost)),
                    ("T desc proxy", np.argsort(-T))):
    mx, mean = sim(order)
    print("%-16s makespan %.3g cycles (%.3f ms at 2.1 GHz), mean %.3f ms, tail %.3f ms" % (name, mx, mx / 2.1e6, mean / 2.1e6, (mx - mean) / 2.1e6))
print("max query cost %.3g cycles (%.3f ms), top-5 %s" % (cost.max(), cost.max() / 2.1e6, np.sort(cost)[-5:] / 2.1e6))
