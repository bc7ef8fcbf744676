import sys, json
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
from _mp import run_ranks
rc, res, logs = run_ranks("ddp_model", 2, sys.argv[1], "2")
print("rc", rc)
if rc: print("\n".join(logs)[-3000:])
a, b = res
for s in range(len(a["grads"])):
    for n, x, y in zip(a["names"], a["grads"][s], b["grads"][s]):
        if x != y: print("step", s, "grad differs", n, x, y)
for n, x, y in zip(a["names"], a["params"], b["params"]):
    if x != y: print("param differs", n, x, y)
