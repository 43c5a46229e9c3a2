"""Debug: run one exchange scenario on the engine and the oracle, report the
first tick whose counters or state differ, field by field."""
import json
import sys

import numpy as np

sys.path[:0] = ["go-libp2p-pubsub_amd", "oracle", "tests"]
import gossip_cases as gc  # noqa: E402
import gsx  # noqa: E402
import oracle as orc  # noqa: E402

kw = json.loads(sys.argv[1])
T = kw.get("T", 2)
g = gc.exchange_run(gsx.Engine(T), **kw)
w = gc.exchange_run(orc.Oracle(T), **kw)
for k in range(len(g[1])):
    diff = {x: (g[1][k][x], w[1][k][x]) for x in g[1][k] if g[1][k][x] != w[1][k][x]}
    bad = []
    for f in g[2][k]:
        a, b = np.atleast_1d(np.asarray(g[2][k][f])), np.atleast_1d(np.asarray(w[2][k][f]))
        if a.shape != b.shape or not np.array_equal(a.view(np.uint8), b.view(np.uint8)):
            idx = np.nonzero(a.reshape(-1) != b.reshape(-1))[0]
            bad.append((f, len(idx), idx[:6].tolist(), a.reshape(-1)[idx[:6]].tolist(), b.reshape(-1)[idx[:6]].tolist()))
    if diff or bad:
        print("tick", k, "counters", diff)
        for x in bad:
            print("  ", x)
        break
else:
    print("all ticks equal")
