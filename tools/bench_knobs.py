"""bench.py with tools/knobs.py's environment switches applied first (experiment runs only):

    PCST_KNN_OVERLAP=0 python tools/bench_knobs.py --steps 10 ...

Counter passes (rocprofv3 --pmc) serialise the dispatches of all queues, so the overlapped step's
cross-stream flag waits would spin until their poll bound: PMC runs use the single-stream layout."""
import os
import runpy
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import knobs  # noqa: E402

knobs.apply()
sys.argv = [os.path.join(os.path.dirname(HERE), "bench.py")] + sys.argv[1:]
runpy.run_path(sys.argv[0], run_name="__main__")
