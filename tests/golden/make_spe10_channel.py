"""Extract the parametric SPE10 test case data (the 105 channel boxes + values and the 3 force boxes of
dune/hdd/linearelliptic/testcases/spe10.hh:31-251) into spe10_parametric_channel.json.

Run in the build container only (it reads /root/reference as text); the JSON is the committed fixture the
tests and the oracle load (the GPU box has no /root/reference)."""
import json
import os
import re

SRC = "/root/reference/dune/hdd/linearelliptic/testcases/spe10.hh"


def parse(text, key):
    dom = {int(m.group(1)): [float(x) for x in re.split(r"[ ;]+", m.group(2).strip())]
           for m in re.finditer(r'"%s\.(\d+)\.domain = \[([^\]]*)\]' % key, text)}
    val = {int(m.group(1)): float(m.group(2)) for m in re.finditer(r'"%s\.(\d+)\.value = ([-0-9.eE+]+)' % key, text)}
    out = []
    for k in sorted(dom):
        lx, ux, ly, uy = dom[k]          # "domain = [x0 x1; y0 y1]" (problems/spe10.hh:198-202)
        out.append([lx, ly, ux, uy, val[k]])
    return out


if __name__ == "__main__":
    text = open(SRC).read()
    data = {"source": "dune/hdd/linearelliptic/testcases/spe10.hh:31-251 (box = lx, ly, ux, uy, value)",
            "channel": parse(text, "channel"), "force": parse(text, "forces")}
    assert len(data["channel"]) == 105 and len(data["force"]) == 3
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "spe10_parametric_channel.json")
    json.dump(data, open(path, "w"), indent=0)
    print(path, len(data["channel"]), len(data["force"]))
