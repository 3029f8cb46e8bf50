"""Program / statement-block structure produced by the compiler and executed by
the runtime (reference: parser/StatementBlock.java + runtime/controlprogram/
{Program,ProgramBlock,IfProgramBlock,WhileProgramBlock,ForProgramBlock,
ParForProgramBlock,FunctionProgramBlock}.java).  The compiler attaches HOP DAG
roots; lops.py turns them into flat instruction lists."""
from __future__ import annotations

from typing import List, Optional


class Block:
    pos = None


class BasicBlock(Block):
    def __init__(self):
        self.roots = []          # ordered sinks + twrites
        self.env_out = {}        # var -> hop at block end (assignments)
        self.reads = set()       # variables transiently read (gen)
        self.writes = set()      # variables assigned (kill)
        self.live_out = set()
        self.rmvars = []         # variables dead after this block
        self.instrs = None
        self.nslots = 0
        self.pos = None
        self.recompile = False

    def __repr__(self):
        return f"BasicBlock(reads={sorted(self.reads)}, writes={sorted(self.writes)})"


class Predicate:
    """A small DAG producing one scalar (if/while predicate, for bounds)."""

    def __init__(self, root, reads):
        self.root = root
        self.reads = set(reads)
        self.instrs = None
        self.nslots = 0
        self.const = root.p["v"] if root.op == "lit" else None
        self.is_const = root.op == "lit"


class IfBlock(Block):
    def __init__(self, pred: Predicate, then_blocks, else_blocks, pos=None):
        self.pred = pred
        self.then_blocks = then_blocks
        self.else_blocks = else_blocks
        self.pos = pos


class WhileBlock(Block):
    def __init__(self, pred: Predicate, body, pos=None):
        self.pred = pred
        self.body = body
        self.pos = pos


class ForBlock(Block):
    def __init__(self, var, start: Predicate, end: Predicate, incr: Optional[Predicate], body,
                 parfor=False, params=None, pos=None):
        self.var = var
        self.start = start
        self.end = end
        self.incr = incr
        self.body = body
        self.parfor = parfor
        self.params = params or {}
        self.pos = pos
        self.result_vars = []     # parfor: variables written in body and live after
        self.accumulators = []    # parfor: result variables only updated by `+=` (summed on merge)


class FunctionBlock(Block):
    def __init__(self, name, namespace, inputs, outputs, body, external=False, ext_params=None, pos=None):
        self.name = name
        self.namespace = namespace
        self.inputs = inputs      # list of ast.Param
        self.outputs = outputs
        self.body = body
        self.external = external
        self.ext_params = ext_params or {}
        self.pos = pos
        self.default_preds = {}   # param name -> Predicate for default value
        self.recursive = False


class CompiledProgram:
    def __init__(self, blocks: List[Block], functions: dict, source=""):
        self.blocks = blocks
        self.functions = functions     # (ns, name) -> FunctionBlock
        self.source = source
        self.inputs = set()            # variables live-in to the program
        self.outputs = set()

    def get_function(self, ns, name):
        return self.functions.get((ns or ".defaultNS", name))
