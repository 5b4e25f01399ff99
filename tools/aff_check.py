import os, sys
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
print("before", len(os.sched_getaffinity(0)), flush=True)
import quant_amd
eng = quant_amd.Engine(0)
print("after engine", len(os.sched_getaffinity(0)), sorted(os.sched_getaffinity(0))[:20], flush=True)
import threading
print("threads", threading.active_count(), flush=True)
