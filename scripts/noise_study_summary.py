"""Summary of scripts/noise_study.py runs against the reference's noise-study table (template.tex:238-279).

Per protocol and noise: the best checkpoint of each run (min(WR_strong, WR_weak) with model_manager's +0.01 rule),
re-evaluated on 1 000 fresh placements per bot (``final_eval``), as mean +- std over seeds (np.std with ddof=1, the
sample standard deviation; the report does not say which it used, ddof=0 is listed too), and Welch's z against the
reference's three-seed mean +- std:  z = (m - m_ref) / sqrt(s^2 / n + s_ref^2 / 3).  Win rates in percent.
With the reference's n = 3 the statistic is Student-t with the Welch-Satterthwaite degrees of freedom (often 2-5),
not normal, so each row also carries ``welch_df`` and the two-sided t-based ``welch_p``
(scipy.stats.ttest_ind_from_stats, equal_var=False); quote p, not a normal cutoff on z.

Usage: python scripts/noise_study_summary.py <dir>... > profiles/r05/noise_study_summary.json
"""
import glob
import json
import math
import os
import sys

import numpy as np

KEYS = (("wr_weak", 100.0), ("wr_strong", 100.0), ("r_weak", 1.0), ("r_strong", 1.0))


def load(dirs):
    runs = {}
    for d in dirs:
        for f in sorted(glob.glob(os.path.join(d, "*_s*.json"))):
            r = json.load(open(f))
            if "final_eval" not in r or r.get("reference") is None:  # stage1: no report table (reference_loop_compare.py)
                continue
            label = r["noise"] if r["protocol"] != "sp_per" else f"per{int(r['per'])}_sp{int(r['self_play'])}"
            runs[(r["protocol"], label, r["seed"])] = r  # later directories override earlier partial runs
    return runs


def welch_df_p(m1, s1, n1, m2, s2, n2):
    """Welch-Satterthwaite degrees of freedom and the two-sided t-test p of two samples given as mean / sample std / n."""
    from scipy.stats import ttest_ind_from_stats

    a, b = s1 ** 2 / n1, s2 ** 2 / n2
    if a + b <= 0 or n1 < 2:
        return None, None
    df = (a + b) ** 2 / (a ** 2 / (n1 - 1) + b ** 2 / (n2 - 1))
    return float(df), float(ttest_ind_from_stats(m1, s1, n1, m2, s2, n2, equal_var=False).pvalue)


def main():
    runs = load(sys.argv[1:])
    out = {"source": "scripts/noise_study.py + scripts/noise_study_summary.py", "reference": "latex/report/template.tex:238-279",
           "protocols": {}}
    for proto in sorted({k[0] for k in runs}):
        pr = {}
        labels = sorted({k[1] for k in runs if k[0] == proto})
        for noise in labels:
            rs = [runs[k] for k in sorted(runs) if k[0] == proto and k[1] == noise]
            if not rs:
                continue
            row = {"seeds": [r["seed"] for r in rs], "n": len(rs)}
            for key, scale in KEYS:
                v = np.array([r["final_eval"][key] * scale for r in rs])
                m, sd1 = float(v.mean()), float(v.std(ddof=1)) if len(v) > 1 else 0.0
                rm, rsd = rs[0]["reference"][key]
                se = math.sqrt(sd1 ** 2 / len(v) + rsd ** 2 / 3)
                df, p = welch_df_p(m, sd1, len(v), rm, rsd, 3)
                row[key] = {"values": [round(float(x), 3) for x in v], "mean": round(m, 3), "std": round(sd1, 3),
                            "std_ddof0": round(float(v.std()), 3), "reference": [rm, rsd],
                            "welch_z": round((m - rm) / se, 2) if se > 0 else None,
                            "welch_df": None if df is None else round(df, 2), "welch_p": None if p is None else round(p, 4)}
            row["selected_at"] = [{"seed": r["seed"], "episode": r["best"]["episode"], "score": r["best"]["score"]}
                                  for r in rs]
            row["all_learned"] = bool(all(r["final_eval"]["wr_weak"] >= 0.85 for r in rs))
            pr[noise] = row
        out["protocols"][proto] = pr
    print(json.dumps(out, indent=1))
    for proto, pr in out["protocols"].items():
        for noise, row in pr.items():
            print(f"{proto:8s} {noise:9s} n={row['n']} " + "  ".join(
                f"{k} {row[k]['mean']:6.2f}+-{row[k]['std']:5.2f} (ref {row[k]['reference'][0]}+-{row[k]['reference'][1]}, "
                f"z {row[k]['welch_z']}, df {row[k]['welch_df']}, p {row[k]['welch_p']})" for k, _ in KEYS), file=sys.stderr)


if __name__ == "__main__":
    main()
