"""Means of a tools/ab_mix.sh log: one line per (scene, build, environment) with its Msamples/s runs.

python tools/ab_summary.py gpurun_out/<tag>/ab_mix.log [more logs]
"""
import collections
import sys


def summarise(paths):
    runs = collections.defaultdict(list)
    for path in paths:
        for line in open(path):
            if "[" not in line or "]" not in line:
                continue
            head, _, rest = line.partition("[")
            env, _, tail = rest.partition("]")
            fields = head.split()
            tail = tail.split()
            if len(fields) < 2 or len(tail) < 2:
                continue
            runs[(tail[0], fields[1], env)].append(float(tail[1]))
    out = []
    for (scene, build, env), v in sorted(runs.items()):
        out.append(f"{scene:16s} {build:10s} [{env}] mean {sum(v) / len(v):10.1f}  runs {v}")
    return out


if __name__ == "__main__":
    print("\n".join(summarise(sys.argv[1:])))
