import sys, json
for l in open(sys.argv[1]):
    if not l.startswith("{"):
        print(l.rstrip()); continue
    d = json.loads(l)
    print(f"{d['test']:22s} {d['mode']:5s} cpi={d['cycles_per_instr']:6.3f} Tops={d['Tops']:6.2f} ms={d['ms']:7.3f} ghz={d['clock_GHz']:.3f}")
