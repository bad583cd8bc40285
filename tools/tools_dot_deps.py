"""Dependency structure of a captured step's HIP graph from its hipGraphDebugDotPrint dump
(tools/tools_capture_dot.py): roots, leaves, and every node whose predecessors are not just the
node captured before it (the forks and joins).

    python tools/tools_dot_deps.py gpurun_out/r04_h/step_split1.dot
"""
import re
import sys
from collections import defaultdict


def parse(path):
    txt = open(path).read()
    nodes = {}
    for m in re.finditer(r'"graph_0_node_(\d+)"\[[^\]]*?label="\{\s*(\w+)(.*?)\}"\];', txt, re.S):
        i, kind, body = int(m.group(1)), m.group(2), m.group(3)
        name = ""
        k = re.search(r"\{ID \| \d+ \| ([^\\<|]+)", body)
        if k:
            name = k.group(1).strip()
        g = re.search(r"\\<\\<\\<\((\d+),(\d+),(\d+)\)", body)
        nodes[i] = (kind, name, g.group(0)[6:].replace("\\", "") if g else "")
    edges = [(int(a), int(b)) for a, b in re.findall(r'"graph_0_node_(\d+)" -> "graph_0_node_(\d+)"', txt)]
    return nodes, edges


def short(name):
    m = re.match(r"_ZN3mrg\d+(\w+?)(E|I)", name)
    if m:
        return m.group(1)
    return name[:40]


def main(path):
    nodes, edges = parse(path)
    pred, succ = defaultdict(list), defaultdict(list)
    for a, b in edges:
        pred[b].append(a)
        succ[a].append(b)
    kinds = defaultdict(int)
    for k, _, _ in nodes.values():
        kinds[k] += 1
    print(f"{path}: {len(nodes)} nodes {dict(kinds)}, {len(edges)} edges")
    print("roots:", [(i, short(nodes[i][1])) for i in sorted(nodes) if not pred[i]])
    print("leaves:", [(i, short(nodes[i][1])) for i in sorted(nodes) if not succ[i]])
    for i in sorted(nodes):
        p = sorted(pred[i])
        if p != [i - 1]:
            print(f"  {i:4d} {nodes[i][0][:6]} {short(nodes[i][1]):32s} {nodes[i][2]:18s} preds {p} succs {sorted(succ[i])}")


if __name__ == "__main__":
    main(sys.argv[1])
