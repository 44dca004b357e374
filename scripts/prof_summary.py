"""Summarise a rocprofv3 kernel_stats.csv: top kernels, grouped by family, per-step ms."""
import argparse
import csv
import re
from collections import defaultdict

FAMILIES = [
    ("hip_conv_fwd/dgrad", r"conv_fwd_kernel|conv_fwd_pipe_kernel|flip_transpose|conv3x3_halo|c1x1_kernel|conv1x1_pers|conv_p8_kernel|conv3x3_hx32|hx32_pack|flip_batch"),
    ("hip_conv_wgrad", r"conv_wgrad_kernel|conv_wgrad_pipe_kernel|conv_wgrad_p8_kernel|wgrad_halo|wgrad3x3_c64|wgrad_reduce|colsum"),
    ("hip_stem", r"stem_"), ("hip_conv_fp8", r"f8|fp8"),
    ("miopen_conv_fwd", r"igemm_fwd|conv_fwd_nhwc|grouped_conv_fwd"), ("miopen_conv_bwd", r"igemm_bwd|bwd_data"),
    ("miopen_conv_wrw", r"igemm_wrw|bwd_weight"), ("relu_bwd/epilogue", r"relu_bwd|bias_res_act|bias_grad"),
    ("losses/targets", r"focal|smooth_l1|anchor_target"), ("adam/norm", r"adam|norm|scale_inplace|refresh"),
    ("pool/upsample", r"maxpool|upsample"), ("torch elementwise", r"at::native"), ("rccl", r"nccl|rccl"),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--steps", type=int, default=1, help="steps covered by the trace (per-step ms)")
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    fam = defaultdict(float)
    for r in rows:
        t = float(r["TotalDurationNs"])
        for name, pat in FAMILIES:
            if re.search(pat, r["Name"]):
                fam[name] += t
                break
        else:
            fam["other"] += t
    print("total GPU kernel time {:.2f} ms over {} steps = {:.2f} ms/step".format(tot / 1e6, a.steps,
                                                                                   tot / 1e6 / a.steps))
    for k, v in sorted(fam.items(), key=lambda kv: -kv[1]):
        print("  {:20s} {:8.2f} ms/step {:5.1f}%".format(k, v / 1e6 / a.steps, 100 * v / tot))
    print("top kernels:")
    for r in rows[:a.top]:
        print("  {:8.2f} ms {:5.1f}% n={:>5} {}".format(float(r["TotalDurationNs"]) / 1e6, float(r["Percentage"]),
                                                       r["Calls"], r["Name"][:120]))


if __name__ == "__main__":
    main()
