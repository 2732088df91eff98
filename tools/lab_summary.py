import sys, json
for l in open(sys.argv[1]):
    d = json.loads(l)
    if "summary" in d:
        print(d["shape"], {k: (v["median"], v.get("ratio_vs_hipblaslt_median")) for k, v in d["summary"].items()})
    elif "bitwise_equal_to_first" in d:
        print(d["shape"], "bitwise", d["bitwise_equal_to_first"])
