import json,sys
for l in open(sys.argv[1]):
    r=json.loads(l)
    print(f"{r['shape']:8s} M={r['M']:5d} q32={r['q32_us']:8.1f} qmm_auto={r['qmm_auto_us']:8.1f} {r['qmm_auto_cfg']} best={r.get('qmm_best_us',0):8.1f} {r.get('qmm_best_cfg')} dense={r['dense_us']:8.1f} TF={r['qmm_tflops']:6.0f} wTB={r['qmm_wTBps']:.2f} err={r.get('qmm_max_rel_err')}")
