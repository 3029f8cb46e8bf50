"""Cross-block speculative fusion: a product computed in a conditional block from a value
that an earlier block produced is evaluated, speculatively, inside that earlier block's
fused pass when the fusion makes it (almost) free.

Motivating case, the trust-region step of MultiLogReg (reference
scripts/algorithms/MultiLogReg.dml:256-264 and :310-314):

    LT = cbind(X %*% B_new, 0); ...; P_new = exp(LT) / rowSums(exp(LT)); obj_new = ...
    ...
    if (is_rho_accepted) {
        P = P_new
        Grad = t(X) %*% (P[, 1:K] - Y[, 1:K])       # second pass over X, on acceptance
    }

The candidate evaluation already streams X once (X %*% B_new, softmax, objective terms:
compiler op `smobj`, rewrites.fuse_softmax_grad); the gradient at the candidate point is
one more MFMA product over the rows that pass holds in registers.  This pass copies the
accept-branch product into the evaluation block as a new variable (`_spec<n>`) computed
from P_new directly, and the branch reads that variable instead.  The copy is kept only if
the earlier block's fusion absorbs it (a trial rewrite of that block must produce a fused
softmax operator that outputs it); otherwise nothing changes, so an unfused backend never
pays an extra pass for a rejected step.

Validity: the branch block reads P_new through a plain copy (`P = P_new`), and neither
P_new nor any other variable the product reads is assigned between the two blocks (the
blocks in between, the branch's predicate and the branch's earlier blocks).  The
speculative value is pure, so evaluating it on a path that never reads it only costs work.
(The reference's codegen has no cross-block fusion; this is a statement-block rewrite in
the style of hops/rewrite/RewriteHoistLoopInvariantOperations.)
"""
from __future__ import annotations

import copy
import itertools

from . import hops as H
from .hops import Hop
from .blocks import BasicBlock, IfBlock, WhileBlock, ForBlock
from .loops import assigned_in, _pure

_names = itertools.count(1)
SPEC_ROW = __import__("os").environ.get("SYSML_SPEC_ROW", "0") == "1"


def _treads(root):
    return {h.p["name"] for h in H.walk([root]) if h.op == "tread"}


def _candidates(bb2):
    """(product hop, source variable of P) for every `t(X) %*% (P[...] - ...)` product in
    bb2's DAG whose P operand is a plain copy of another variable."""
    out = []
    for h in H.walk(list(bb2.roots) + list(bb2.env_out.values())):
        if h.op != "mm" or not h.inputs or h.inputs[0].op != "t":
            continue
        g = h.inputs[1]
        if g.op != "b" or g.p.get("o") != "-" or g.inputs[0].op != "rix":
            continue
        src = g.inputs[0].inputs[0]
        if src.op != "tread":
            continue
        if not all(_pure(x) for x in H.walk([h])):
            continue
        out.append((h, src.p["name"]))
    return out


def _substitute(bb2, old, new):
    for h in H.walk(list(bb2.roots) + list(bb2.env_out.values())):
        if any(c is old for c in h.inputs):
            h.inputs = [new if c is old else c for c in h.inputs]
    bb2.roots = [new if r is old else r for r in bb2.roots]
    bb2.env_out = {k: (new if v is old else v) for k, v in bb2.env_out.items()}


def _clone_into(root, bb1, src_var):
    """Copy the DAG of `root` into bb1's DAG: transient reads of src_var become bb1's value
    of it, every other transient read a read in bb1 (None if bb1 assigns that variable)."""
    memo = {}
    reads = {}
    for h in H.walk(list(bb1.roots) + list(bb1.env_out.values())):
        if h.op == "tread" and h.p["name"] not in reads:
            reads[h.p["name"]] = h

    def cl(h):
        r = memo.get(h.id)
        if r is not None:
            return r
        if h.op == "tread":
            n = h.p["name"]
            if n == src_var:
                r = bb1.env_out[n]
            elif n in bb1.writes:
                raise LookupError(n)
            else:
                r = reads.get(n)
                if r is None:
                    r = Hop("tread", p=dict(h.p), dt=h.dt, dim1=h.dim1, dim2=h.dim2, pos=h.pos)
                    reads[n] = r
        elif h.op == "lit":
            r = h
        else:
            r = Hop(h.op, [cl(c) for c in h.inputs], dict(h.p), named=list(h.named), dt=h.dt,
                    dim1=h.dim1, dim2=h.dim2, pos=h.pos)
        memo[h.id] = r
        return r
    return cl(root)


def _fuses(bb1, var, config):
    """Trial rewrite of a copy of bb1: does the speculative product end up as an output of
    a fused pass over X (smobj / smgrad, or a multi-output Row-template program)?"""
    from . import rewrites as RW
    trial = copy.deepcopy(bb1)
    trial.live_out = None
    RW.rewrite_block(trial, config)
    h = trial.env_out.get(var)
    # absorbed by the hand-matched softmax pass, or (SYSML_SPEC_ROW=1) an output of a merged
    # multi-output Row program that streams X anyway (codegen.merge_row_programs).  The latter
    # is off by default: measured on the MI355X, the generated kernel that adds t(X) %*% W to
    # the candidate pass (VALU register accumulators) is slower than the separate MFMA product
    # on acceptance (MultiLogReg 10M x 1K: 520 vs 461 ms/step with the softmax matcher off)
    return h is not None and h.op == "fout" and (h.inputs[0].op in ("smobj", "smgrad") or
                                                  (SPEC_ROW and h.inputs[0].op == "row" and h.inputs[0].p["prog"].more))


def _try_pair(bb1, mid_writes, bb2, config, stats):
    for prod, pvar in _candidates(bb2):
        if pvar not in bb1.env_out or pvar in mid_writes:
            continue
        if (_treads(prod) - {pvar}) & (mid_writes | bb1.writes):
            continue
        try:
            clone = _clone_into(prod, bb1, pvar)
        except LookupError:
            continue
        var = f"_spec{next(_names)}"
        bb1.env_out[var] = clone
        bb1.writes.add(var)
        if not _fuses(bb1, var, config):
            del bb1.env_out[var]
            bb1.writes.discard(var)
            continue
        for r in H.walk([clone]):
            if r.op == "tread":
                bb1.reads.add(r.p["name"])
        _substitute(bb2, prod, Hop("tread", p={"name": var}, dt=prod.dt, dim1=prod.dim1, dim2=prod.dim2,
                                   pos=prod.pos))
        bb2.reads.add(var)
        stats["speculative-fused-products"] = stats.get("speculative-fused-products", 0) + 1


def _scan(blocks, config, stats):
    for k, b in enumerate(blocks):
        if isinstance(b, IfBlock):
            _scan(b.then_blocks, config, stats)
            _scan(b.else_blocks, config, stats)
        elif isinstance(b, (WhileBlock, ForBlock)) and not (isinstance(b, ForBlock) and b.parfor):
            _scan(b.body, config, stats)
        if not isinstance(b, BasicBlock) or not b.env_out:
            continue
        # later if-blocks of this list whose first then-block is a basic block
        mid = set()
        for j in range(k + 1, len(blocks)):
            c = blocks[j]
            if isinstance(c, IfBlock) and c.then_blocks and isinstance(c.then_blocks[0], BasicBlock):
                _try_pair(b, mid, c.then_blocks[0], config, stats)
            mid |= assigned_in([c])


def run(cp, config=None):
    """Apply to the main program and every function body; returns rewrite counters."""
    if config is not None and not (getattr(config, "rewrites", True) and getattr(config, "fusion", True)):
        return {}
    stats = {}
    _scan(cp.blocks, config, stats)
    for fb in cp.functions.values():
        if fb.body is not None:
            _scan(fb.body, config, stats)
    return stats
