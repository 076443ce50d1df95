#!/usr/bin/env python3
"""Extract offline data tables and golden vectors from the reference checkout.

Runs HERE only (needs /root/reference); its outputs are committed so that nothing
on the GPU box ever reads the reference. Everything written is DATA (inputs and
expected outputs), never reference source text.

Outputs
  karpenter-provider-aws_amd/data/ec2_instance_types.tsv
      EC2 DescribeInstanceTypes-shaped facts per type, reconstructed from
      R:website/content/en/preview/reference/instance-types.md (labels),
      R:pkg/providers/instancetype/zz_generated.vpclimits.go (ENI limits) and
      R:pkg/providers/pricing/zz_generated.pricing_aws.go:25 (us-east-1 OD price).
  tests/golden/docs_allocatable.tsv
      The docs' *allocatable* resources per type (generated upstream by
      R:hack/docs/instancetypes_gen/main.go:129-266 with AL2023, no BDMs,
      VMMemoryOverheadPercent=0.075) -- the golden vector for types.go.
  tests/golden/docs_labels.tsv
      The docs' single-valued labels per type (golden for computeRequirements).
"""
import os
import re
import sys

REF = "/root/reference"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DOCS = f"{REF}/website/content/en/preview/reference/instance-types.md"
VPC = f"{REF}/pkg/providers/instancetype/zz_generated.vpclimits.go"
PRICE = f"{REF}/pkg/providers/pricing/zz_generated.pricing_aws.go"

BIN = {"Ki": 1 << 10, "Mi": 1 << 20, "Gi": 1 << 30, "Ti": 1 << 40}
DEC = {"k": 10**3, "M": 10**6, "G": 10**9, "T": 10**12}


def qty_milli(s):
    """k8s quantity string -> integer milli-units (exact)."""
    m = re.fullmatch(r"(-?\d+)(m|Ki|Mi|Gi|Ti|k|M|G|T)?", s)
    if not m:
        raise ValueError(s)
    n, suf = int(m.group(1)), m.group(2)
    if suf is None:
        return n * 1000
    if suf == "m":
        return n
    if suf in BIN:
        return n * BIN[suf] * 1000
    return n * DEC[suf] * 1000


def parse_docs():
    types = []
    cur = None
    section = None
    for line in open(DOCS):
        line = line.rstrip("\n")
        m = re.match(r"^### `([^`]+)`", line)
        if m:
            cur = {"name": m.group(1), "labels": {}, "res": {}}
            types.append(cur)
            section = None
            continue
        if line.startswith("#### Labels"):
            section = "labels"
            continue
        if line.startswith("#### Resources"):
            section = "res"
            continue
        if cur is None or section is None:
            continue
        m = re.match(r"^ \|([^|]+)\|([^|]*)\|$", line)
        if not m or m.group(1).strip() in ("Label", "Resource", "--"):
            continue
        k, v = m.group(1), m.group(2)
        if section == "labels":
            cur["labels"][k] = v
        else:
            cur["res"][k] = v
    return types


def parse_vpclimits():
    src = open(VPC).read()
    out = {}
    for m in re.finditer(r'\n\t"([^"]+)": \{(.*?)\n\t\},', src, re.S):
        name, body = m.group(1), m.group(2)

        def f(field):
            mm = re.search(rf"\b{field}:\s+([^,\n]+),", body)
            return mm.group(1).strip() if mm else None

        dflt = int(f("DefaultNetworkCardIndex"))
        cards = [(int(a), int(b)) for a, b in re.findall(
            r"MaximumNetworkInterfaces:\s+(\d+),\s+NetworkCardIndex:\s+(\d+),", body)]
        card_max = {idx: mx for mx, idx in cards}
        out[name] = {
            "interface": int(f("Interface")),
            "ipv4": int(f("IPv4PerInterface")),
            "trunk": f("IsTrunkingCompatible") == "true",
            "branch": int(f("BranchInterface")),
            "default_card_max": card_max.get(dflt, int(f("Interface"))),
        }
    return out


def parse_prices():
    src = open(PRICE).read()
    start = src.index('"us-east-1": {')
    end = src.index("\n\t},", start)
    body = src[start:end]
    return {k: float(v) for k, v in re.findall(r'"([a-z0-9\-.]+)":\s*([0-9.]+)', body) if k != "us-east-1"}


def main():
    docs = parse_docs()
    vpc = parse_vpclimits()
    prices = parse_prices()
    assert len(docs) == 919, len(docs)
    data_dir = os.path.join(REPO, "karpenter-provider-aws_amd", "data")
    gold_dir = os.path.join(REPO, "tests", "golden")
    os.makedirs(data_dir, exist_ok=True)
    os.makedirs(gold_dir, exist_ok=True)

    cols = ["name", "vcpu", "memory_mib", "arch", "hypervisor", "encryption_in_transit",
            "cpu_manufacturer", "clock_mhz", "ebs_bandwidth", "network_bandwidth", "local_nvme_gb",
            "gpu_name", "gpu_manufacturer", "gpu_count", "gpu_memory_mib",
            "accel_name", "accel_manufacturer", "accel_count", "neuron_devices", "neuron_cores_per_device",
            "efa", "max_enis", "ipv4_per_eni", "trunking", "branch_enis", "eni_source", "od_price"]
    rows = []
    n_inferred = 0
    for t in docs:
        L, R = t["labels"], t["res"]
        g = lambda k: L.get("karpenter.k8s.aws/" + k, "")
        name = t["name"]
        neuron = qty_milli(R["aws.amazon.com/neuron"]) // 1000 if "aws.amazon.com/neuron" in R else 0
        ncores = qty_milli(R["aws.amazon.com/neuroncore"]) // 1000 if "aws.amazon.com/neuroncore" in R else 0
        efa = qty_milli(R["vpc.amazonaws.com/efa"]) // 1000 if "vpc.amazonaws.com/efa" in R else 0
        if name in vpc:
            v = vpc[name]
            enis, ipv4, trunk, branch, src = v["default_card_max"], v["ipv4"], int(v["trunk"]), v["branch"], "vpclimits"
        else:
            # Not in the limits table: the reference takes ENI facts from live EC2 data we do not
            # have. Reconstruct a (1 ENI, pods-1 IPv4) pair that reproduces the docs' pod count
            # through ENILimitedPods (R:types.go:461-475); pod-eni stays 0 as in R:types.go:388-395.
            pods = qty_milli(R["pods"]) // 1000
            enis, ipv4, trunk, branch, src = 1, pods - 1, 0, 0, "inferred_from_docs_pods"
            n_inferred += 1
        rows.append([
            name, L["karpenter.k8s.aws/instance-cpu"], L["karpenter.k8s.aws/instance-memory"],
            L["kubernetes.io/arch"], g("instance-hypervisor"),
            g("instance-encryption-in-transit-supported") or "false",
            g("instance-cpu-manufacturer"), g("instance-cpu-sustained-clock-speed-mhz"),
            g("instance-ebs-bandwidth"), g("instance-network-bandwidth"), g("instance-local-nvme"),
            g("instance-gpu-name"), g("instance-gpu-manufacturer"), g("instance-gpu-count") or "0",
            g("instance-gpu-memory"), g("instance-accelerator-name"), g("instance-accelerator-manufacturer"),
            g("instance-accelerator-count") or "0", str(neuron),
            str(ncores // neuron if neuron else 0), str(efa), str(enis), str(ipv4), str(trunk), str(branch), src,
            ("%.6f" % prices[name]) if name in prices else "-1",
        ])
    with open(os.path.join(data_dir, "ec2_instance_types.tsv"), "w") as f:
        f.write("# generated by tools/extract_fixtures.py from the reference's offline tables (data only)\n")
        f.write("\t".join(cols) + "\n")
        for r in rows:
            f.write("\t".join(r) + "\n")

    res_names = ["cpu", "memory", "ephemeral-storage", "pods", "vpc.amazonaws.com/pod-eni", "vpc.amazonaws.com/efa",
                 "nvidia.com/gpu", "amd.com/gpu", "aws.amazon.com/neuron", "aws.amazon.com/neuroncore",
                 "habana.ai/gaudi"]
    with open(os.path.join(gold_dir, "docs_allocatable.tsv"), "w") as f:
        f.write("# docs allocatable (R:website/content/en/preview/reference/instance-types.md), milli-units\n")
        f.write("name\t" + "\t".join(res_names) + "\n")
        for t in docs:
            f.write(t["name"] + "\t" + "\t".join(str(qty_milli(t["res"][r])) if r in t["res"] else "0"
                                                 for r in res_names) + "\n")
    with open(os.path.join(gold_dir, "docs_labels.tsv"), "w") as f:
        f.write("# docs single-valued labels (R:website/content/en/preview/reference/instance-types.md)\n")
        f.write("name\tkey\tvalue\n")
        for t in docs:
            for k in sorted(t["labels"]):
                f.write(f"{t['name']}\t{k}\t{t['labels'][k]}\n")
    print(f"types={len(rows)} eni_inferred={n_inferred} priced={sum(1 for t in docs if t['name'] in prices)}")


if __name__ == "__main__":
    sys.exit(main())
