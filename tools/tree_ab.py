"""A/B timing of the broadcast-tree walk (bench.py's noc.broadcast_tree
workload) for the library GG_LIB names (diagnostic builds included)."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402

a = argparse.Namespace(noc_packets=1 << 18, no_verify=True)
r = bench.noc_tree_bench(a, "cuda", 1024)
print(json.dumps({"lib": os.environ.get("GG_LIB", "default"), "seconds": r["seconds"]}))
