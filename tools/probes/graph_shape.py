"""Shape of a captured step graph: node and edge counts, node kinds, and whether it is a straight
line (the ResNet-50 full graph replays node by node -- 2.9 ms of host enqueue
-- with the own RCCL communicator, 0.18 ms with the local one).

    EWDML_GRAPH_DUMP=/tmp/g.dot python bench.py ... ; python tools/probes/graph_shape.py /tmp/g.dot

Reads the DOT file written by hipGraphDebugDotPrint (torch CUDAGraph.debug_dump)."""
import collections
import re
import sys


def shape(path):
    txt = open(path).read()
    nodes = {}
    for m in re.finditer(r'^\s*"?(\w+)"?\s*\[(.*?)\];?\s*$', txt, re.M):
        name, attrs = m.group(1), m.group(2)
        if name in ("graph", "node", "edge"):
            continue
        lab = re.search(r'label="(.*?)"', attrs, re.S)
        nodes[name] = lab.group(1) if lab else attrs
    edges = re.findall(r'"?(\w+)"?\s*->\s*"?(\w+)"?', txt)
    outd, ind = collections.Counter(a for a, _ in edges), collections.Counter(b for _, b in edges)
    kinds = collections.Counter()
    for lab in nodes.values():
        k = re.split(r"[\\\n|{}: ]+", lab.strip("{} "))
        kinds[next((w for w in k if w), "?")[:40]] += 1
    forks = [n for n, d in outd.items() if d > 1]
    joins = [n for n, d in ind.items() if d > 1]
    return {"nodes": len(nodes), "edges": len(edges), "forks": len(forks), "joins": len(joins),
            "linear": not forks and not joins, "kinds": kinds.most_common(12),
            "fork_labels": [nodes.get(n, n)[:120] for n in forks[:8]],
            "join_labels": [nodes.get(n, n)[:120] for n in joins[:8]]}


if __name__ == "__main__":
    import json

    for p in sys.argv[1:]:
        print(p, json.dumps(shape(p), indent=1))
