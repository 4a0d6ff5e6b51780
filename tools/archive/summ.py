import json, sys
for line in sys.stdin:
    line = line.strip()
    if line.startswith("{"):
        d = json.loads(line)
        print("value", d["value"], "ms/step", d["ms_per_step"], "dp_ms", d["roofline"]["kernel_ms"],
              "finish_ms", d["roofline"]["finish_ms"], "cpu", d.get("cpu_baseline") and d["cpu_baseline"]["value"])
    else:
        print(line[:400])
