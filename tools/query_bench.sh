#!/bin/bash
# Per-packet query throughput of the drop-in on the GPU box (tools/query_bench.c).
set -o pipefail
mkdir -p gpurun_out
W=$(mktemp -d /tmp/qb.XXXXXX)
python - "$W" <<'PY'
import lzma, sys
sys.path.insert(0, ".")
from shadow_amd.routes import Graph
from tests.util import write_graphml
w = sys.argv[1]
open(f"{w}/full.graphml.xml", "wb").write(lzma.open("tests/golden/topologies/topology.graphml.xml.xz").read())
g = Graph.generate("ba", 100000, 3, 1)
ef, et, lat, lo, vl = g.export()
write_graphml(f"{w}/ba100k.graphml.xml", g.V, ef, et, lat, lo, vl)
print("graphs written", flush=True)
PY
for t in 1 16; do timeout -k 10 120 ./tools/query_bench $W/full.graphml.xml 1000 500000 $t || exit 9; done
for t in 1 16; do timeout -k 10 120 ./tools/query_bench $W/ba100k.graphml.xml 5000 500000 $t || exit 9; done
rm -rf "$W"
