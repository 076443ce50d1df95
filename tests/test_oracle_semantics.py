"""Requirements algebra of the oracle against the upstream semantics written in SURVEY §8(a) a10
(scheduling.Requirement Intersection / Len / Operator / Intersects / Compatible). These pin the oracle's
restatement of sigs.k8s.io/karpenter behaviour that the reference's own tests exercise through
R:pkg/providers/instancetype/suite_test.go (e.g. NotIn / DoesNotExist exemptions, Gt/Lt bounds)."""
import pytest

from oracle import pyoracle as O

Z = "topology.kubernetes.io/zone"
CPU = "karpenter.k8s.aws/instance-cpu"
CUSTOM = "example.com/team"


@pytest.mark.parametrize("a,b,expect", [
    ([(Z, "In", ["a"])], [(Z, "In", ["a", "b"])], True),
    ([(Z, "In", ["a"])], [(Z, "In", ["b"])], False),
    ([(Z, "In", ["a"])], [(Z, "NotIn", ["a"])], False),
    ([(Z, "NotIn", ["a"])], [(Z, "NotIn", ["a"])], True),           # empty? no: complement ∪ -> non-empty
    ([(Z, "DoesNotExist", [])], [(Z, "NotIn", ["a"])], True),       # both NotIn/DNE: exempt
    ([(Z, "DoesNotExist", [])], [(Z, "In", ["a"])], False),
    ([(Z, "DoesNotExist", [])], [(Z, "Exists", [])], False),
    ([(CPU, "In", ["4"])], [(CPU, "Gt", ["3"])], True),
    ([(CPU, "In", ["4"])], [(CPU, "Gt", ["4"])], False),
    ([(CPU, "In", ["4"])], [(CPU, "Lt", ["5"])], True),
    ([(CPU, "Gt", ["5"])], [(CPU, "Lt", ["5"])], False),            # gt >= lt -> DoesNotExist
    ([(CPU, "Gt", ["4"])], [(CPU, "Lt", ["6"])], True),             # complement with bounds: Len > 0
    ([(CPU, "In", ["x"])], [(CPU, "Gt", ["1"])], False),            # non-integer values drop under bounds
])
def test_intersects(a, b, expect):
    assert O.requirements_intersects(a, b) is expect
    assert O.requirements_intersects(b, a) is expect


def test_compatible_undefined_keys():
    # custom key undefined on the left: only NotIn/DoesNotExist pass
    assert O.requirements_compatible([], [(CUSTOM, "In", ["a"])]) is False
    assert O.requirements_compatible([], [(CUSTOM, "NotIn", ["a"])]) is True
    assert O.requirements_compatible([], [(CUSTOM, "DoesNotExist", [])]) is True
    # well-known keys are allowed undefined only with AllowUndefinedWellKnownLabels
    assert O.requirements_compatible([], [(Z, "In", ["a"])], allow_wellknown=True) is True
    assert O.requirements_compatible([], [(Z, "In", ["a"])], allow_wellknown=False) is False
    # normalized labels (karpv1.NormalizedLabels)
    assert O.requirements_compatible([(Z, "In", ["a"])], [("failure-domain.beta.kubernetes.io/zone", "In", ["b"])]) is False
