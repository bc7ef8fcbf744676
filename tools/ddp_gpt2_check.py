import sys, os
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
from _mp import run_ranks
for env in ({"PDE_DDP_REDUCE_DTYPE": "param"}, {}):
    rc, res, logs = run_ranks("ddp_model", 2, "gpt2", "3", extra_env=env)
    print(env, rc, res[0]["params"][:3] if res[0] else None, res[1]["params"][:3] if res[1] else None, flush=True)
    print(env, "losses", res[0]["losses"] if res[0] else None, res[1]["losses"] if res[1] else None)
    print(env, "grads0", (res[0]["grads"][0][:4] if res[0] else None), (res[1]["grads"][0][:4] if res[1] else None))
