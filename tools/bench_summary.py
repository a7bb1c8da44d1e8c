"""One-screen summary of a bench.py JSON line (the headline and every leg)."""
import json
import sys


def main():
    d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
    r = d.get("roofline", {})
    print("line bytes %d" % len(json.dumps(d)))
    print("c2 %.4g G/s kernel %.3f ms frac %.4f traffic %s" % (d["value"] / 1e9, r.get("kernel_ms", 0),
                                                                r.get("frac", 0), r.get("traffic")))
    for k, v in (d.get("legs") or {}).items():
        print("  leg %-10s %s" % (k, json.dumps(v)))
    b = d.get("bpe_c3", {})
    if b:
        print("c3 %.4g G/s kernel %.3f ms frac %s traffic %s" % (b.get("value", 0) / 1e9,
                                                               b.get("roofline", {}).get("kernel_ms", 0),
                                                               b.get("roofline", {}).get("frac"),
                                                               b.get("roofline", {}).get("traffic")))
    j = d.get("ja_multibyte", {})
    if j:
        print("ja %.4g M/s coop %s" % (j.get("value", 0) / 1e6, json.dumps(j.get("roofline", {}).get("coop"))))
    e = d.get("estep", {})
    if e:
        print("estep PARITY %s s/epoch roof %s" % (e.get("value"), json.dumps(
            {k: e.get("roofline", {}).get(k) for k in ("kernel_ms", "frac", "traffic")})))
    t = d.get("train", {})
    if t:
        print("c5 %s s peak %s" % (t.get("value"), t.get("peak_device_bytes")))
    tb = d.get("train_bpe", {})
    if tb:
        st = tb.get("stages", {})
        print("bpe train %s s %s" % (tb.get("value"), {k: st.get(k) for k in st if k.startswith("bpe_")}))
    l = d.get("latency", {})
    if l:
        print("latency single %s us batches %s" % (l.get("encode_single_us"),
                                                   [(x["batch"], x["us_per_call"]) for x in l.get("batches", [])][:5]))
        print("c1 botchan %s lines/s" % l.get("c1_botchan", {}).get("line_by_line_sentences_per_s"))
    if d.get("e2e_raw"):
        print("e2e_raw %s" % d["e2e_raw"].get("value"))
    print("parity %s" % {k: (v.get("mismatches") if isinstance(v, dict) else v)
                         for k, v in d.get("parity", {}).items()})


if __name__ == "__main__":
    main()
