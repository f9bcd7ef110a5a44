"""Render a layer graph (reference C31 visualisation, script/graph.py +
script/draw.py, which needed networkx / pygraphviz / matplotlib) as Graphviz
DOT text, from either a node-link JSON file (``NeuralNet.to_json`` /
``Graph::ToJson``: ``{"directed","nodes":[{"id","color","shape"}],"links":
[{"source","target","color"}]}``) or straight from a model conf:

    python tools/draw_graph.py --json graph.json > net.dot
    python tools/draw_graph.py --model_conf examples/mnist/conv.conf [--group_size 2] > net.dot
    dot -Tpng net.dot -o net.png          # wherever Graphviz is installed

Partitions are coloured by ``locationid``; connection layers (slice /
concate / split / bridge) are drawn as ellipses, the rest as boxes -- the
reference's conventions.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

PALETTE = ["black", "red", "blue", "darkgreen", "orange", "purple", "brown", "magenta", "cyan", "gray"]


def to_dot(g: dict, name: str = "net") -> str:
    out = [f'digraph "{name}" {{', "  rankdir=TB;", "  node [fontsize=10];"]
    ids = []
    for n in g.get("nodes", []):
        nid = n["id"]
        ids.append(nid)
        color = n.get("color", "black")
        if isinstance(color, int):
            color = PALETTE[color % len(PALETTE)]
        shape = n.get("shape", "box")
        out.append(f'  "{nid}" [color="{color}", shape="{shape}"];')
    for e in g.get("links", []):
        s, t = e["source"], e["target"]
        s = ids[s] if isinstance(s, int) else s
        t = ids[t] if isinstance(t, int) else t
        color = e.get("color", "black")
        if isinstance(color, int):
            color = PALETTE[color % len(PALETTE)]
        out.append(f'  "{s}" -> "{t}" [color="{color}"];')
    out.append("}")
    return "\n".join(out) + "\n"


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default="", help="node-link JSON file")
    ap.add_argument("--model_conf", default="", help="ModelProto text conf (the train net is built on the CPU)")
    ap.add_argument("--group_size", type=int, default=1, help="partition the net over this many locations")
    a = ap.parse_args(argv)
    if a.json:
        with open(a.json) as f:
            g = json.load(f)
        name = os.path.basename(a.json)
    elif a.model_conf:
        from singa_amd import device
        from singa_amd.config import schema
        from singa_amd.runtime import NeuralNet

        mp = schema.read_text_file("ModelProto", a.model_conf)
        net = NeuralNet(mp.neuralnet, a.group_size, "kTrain", device.get_default_device(),
                        {"*": {"shape": (28, 28), "nclass": 10}})
        g = json.loads(net.to_json())
        name = mp.name or "net"
    else:
        ap.error("give --json or --model_conf")
    sys.stdout.write(to_dot(g, name))
    return 0


if __name__ == "__main__":
    sys.exit(main())
