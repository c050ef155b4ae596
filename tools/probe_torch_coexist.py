import sys, os
sys.path.insert(0, os.getcwd())
order = sys.argv[1]
if order == "torch_first":
    import torch
    print("torch cuda avail", torch.cuda.is_available(), torch.cuda.device_count())
import firedancer_amd as fa
from firedancer_amd import workload
e = fa.VerifyEngine(0, max_txn=1024)
a, t, m = workload.cfg1(512, seed=3)
c = e.verify_txns(a, t)
print(order, "engine ok", ((c == 0) == (m == 0)).all())
if order == "ours_first":
    import torch
    import torch.distributed as dist
    print("torch imported after engine; cuda avail:", torch.cuda.is_available())
e.close()
