"""keto_amd — MI355X-native batched permission checks behind Ory Keto's check and
expand engines.  See DESIGN.md.  Native code: keto_amd/libketogpu.so (C ABI in
include/ketogpu.h), built in-tree by `python -m keto_amd.build`."""
from .relationtuple import InternalRelationTuple, SubjectID, SubjectSet  # noqa: F401

__all__ = ["InternalRelationTuple", "SubjectID", "SubjectSet"]
