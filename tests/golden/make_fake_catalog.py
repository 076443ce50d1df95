"""Extract the reference's fake EC2 offering table (data only) into tests/golden/fake_offerings.tsv.

Source: R:pkg/fake/zz_generated.describe_instance_types.go:888-1003 (defaultDescribeInstanceTypeOfferingsOutput),
the 16-type catalogue the instancetype suite (R:pkg/providers/instancetype/suite_test.go) provisions against.
Each row is (instance type, zone) exactly as the Go literal lists them; no source text is kept.
Run from the repo root with the reference present: python tests/golden/make_fake_catalog.py
"""
import os
import re
import sys

REF = "/root/reference/pkg/fake/zz_generated.describe_instance_types.go"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fake_offerings.tsv")


def main(path=REF):
    text = open(path).read()
    block = text[text.index("defaultDescribeInstanceTypeOfferingsOutput"):]
    pairs = re.findall(r'InstanceType:\s*"([^"]+)",\s*Location:\s*lo\.ToPtr\("([^"]+)"\)', block)
    if not pairs:
        sys.exit("no offerings found")
    with open(OUT, "w") as f:
        f.write("# R:pkg/fake/zz_generated.describe_instance_types.go:888-1003 (extracted by make_fake_catalog.py)\n")
        f.write("instance_type\tzone\n")
        for t, z in pairs:
            f.write(f"{t}\t{z}\n")
    print(f"{len(pairs)} offerings of {len(set(t for t, _ in pairs))} types -> {OUT}")


if __name__ == "__main__":
    main(*sys.argv[1:])
