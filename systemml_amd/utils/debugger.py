"""Interactive DML debugger (reference: org/apache/sysml/debug/{DMLDebugger,DMLDebuggerFunctions,
DMLBreakpointManager,DebugState}.java; enabled by the `-debug` command-line option).

Commands (same spirit as the reference's gdb-like interface):
    r | run                 start / restart execution
    b | break LINE          set a breakpoint on a source line
    d | delete LINE         remove a breakpoint
    i | info                list breakpoints
    c | continue            run to the next breakpoint
    s | step | n | next     execute until the next source line
    p | print VAR           print a variable (matrices: shape + leading cells)
    w | whatis VAR          data / value type and size of a variable
    v | vars                list the live variables of the current frame
    l | list [LINE]         show source lines around LINE (default: current)
    q | quit                abort the program
Breakpoints fire before the first instruction compiled from that line.  Variables are
looked up in the running statement block first (intermediate slots are kept alive in
debug mode), then in the frame's symbol table.
"""
from __future__ import annotations

import sys

import torch

from ..parser.errors import DMLScriptStop


class Debugger:
    def __init__(self, compiled, inp=None, out=None, source=None):
        self.cs = compiled
        self.inp = inp or sys.stdin
        self.out = out or sys.stdout
        self.breakpoints = set()
        self.stepping = False
        self.last_line = None
        self.cur_line = None
        self.ctx = None
        self.src_lines = (source or getattr(compiled, "source", "") or "").split("\n")

    # ------------------------------------------------------------------ I/O
    def _w(self, s):
        self.out.write(s + "\n")
        self.out.flush()

    def _read(self):
        self.out.write("(SystemML-AMD debug) ")
        self.out.flush()
        line = self.inp.readline()
        if not line:
            return "q"
        return line.strip()

    # ------------------------------------------------------------------ driver
    def run(self):
        from ..api import executor as EX
        self._w("SystemML-AMD debugger: r(un), b(reak) N, c(ontinue), s(tep), p(rint) V, l(ist), q(uit)")
        while True:
            cmd = self._read()
            if cmd in ("r", "run"):
                break
            if cmd in ("q", "quit"):
                return None
            self._command(cmd, before_run=True)
        self.stepping = False
        cs = self.cs
        config = cs.config
        if getattr(config, "fusion", False) and getattr(cs, "compile_args", None) is not None:
            # debug mode runs the unfused plan (as the reference's debug mode disables block
            # merging): every statement keeps its own instructions and its variables
            import dataclasses
            config = dataclasses.replace(config, fusion=False)
            cs = self.cs = EX.compile_script(cs.source, config=config, **cs.compile_args)
        EX.backend.configure(config)
        from ..runtime.program import ExecutionContext, exec_blocks
        self._keep_slots(cs.cp)
        self.ctx = ctx = ExecutionContext(cs.cp, config, out=self._w)
        ctx.debugger = self
        try:
            exec_blocks(ctx, cs.cp.blocks)
        except DMLScriptStop as e:
            self._w(f"Program stopped: {e}")
            return ctx
        self._w("Program finished.")
        return ctx

    @staticmethod
    def _keep_slots(cp):
        """Debug mode keeps every intermediate slot alive so variables stay inspectable."""
        from ..compiler.blocks import BasicBlock, IfBlock, WhileBlock, ForBlock

        def visit(blocks):
            for b in blocks:
                if isinstance(b, BasicBlock):
                    for ins in b.instrs or ():
                        ins.free = ()
                elif isinstance(b, IfBlock):
                    visit(b.then_blocks)
                    visit(b.else_blocks)
                elif isinstance(b, (WhileBlock, ForBlock)):
                    visit(b.body)
        visit(cp.blocks)
        for fb in cp.functions.values():
            visit(getattr(fb, "body", []) or [])

    # called by the runtime before each instruction
    def _lookup(self, name):
        """Variable value: already-computed assignments of the running block first."""
        blk, slots = getattr(self, "cur_block", None), getattr(self, "cur_slots", None)
        if blk is not None and slots is not None:
            sl = getattr(blk, "debug_slots", {}).get(name)
            if sl is not None and sl < len(slots) and slots[sl] is not None:
                return True, slots[sl]
        if self.ctx is not None and name in self.ctx.vars:
            return True, self.ctx.vars[name]
        return False, None

    def on_instruction(self, ctx, ins, slots=None):
        self.cur_slots = slots
        hop = getattr(ins, "hop", None)
        pos = getattr(hop, "pos", None)
        line = getattr(pos, "line", None)
        # a fused operator (compiler/codegen.py) covers several source lines: each of them
        # is visited in order, so breakpoints on the fused statements still fire
        lines = list(getattr(hop, "p", {}).get("lines") or ([] if line is None else [line]))
        for line in lines:
            if line == self.last_line:
                continue
            self.last_line = line
            self.cur_line = line
            if self.stepping or line in self.breakpoints:
                self.stepping = False
                self._w(f"Breakpoint at line {line}: {self._src(line)}")
                self._interact(ctx)

    def _interact(self, ctx):
        while True:
            cmd = self._read()
            if cmd in ("c", "continue"):
                return
            if cmd in ("s", "step", "n", "next"):
                self.stepping = True
                return
            if cmd in ("q", "quit"):
                raise DMLScriptStop("debugger quit")
            self._command(cmd)

    # ------------------------------------------------------------------ commands
    def _src(self, line):
        if 1 <= line <= len(self.src_lines):
            return self.src_lines[line - 1].strip()
        return ""

    def _command(self, cmd, before_run=False):
        parts = cmd.split()
        if not parts:
            return
        c, args = parts[0], parts[1:]
        if c in ("b", "break") and args:
            self.breakpoints.add(int(args[0]))
            self._w(f"Breakpoint set at line {args[0]}")
        elif c in ("d", "delete") and args:
            self.breakpoints.discard(int(args[0]))
            self._w(f"Breakpoint at line {args[0]} deleted")
        elif c in ("i", "info"):
            self._w("Breakpoints: " + (", ".join(str(b) for b in sorted(self.breakpoints)) or "none"))
        elif c in ("l", "list"):
            at = int(args[0]) if args else (self.cur_line or 1)
            for k in range(max(1, at - 3), min(len(self.src_lines), at + 3) + 1):
                mark = "=>" if k == self.cur_line else ("b " if k in self.breakpoints else "  ")
                self._w(f"{mark}{k:4d}  {self.src_lines[k - 1]}")
        elif c in ("v", "vars"):
            if self.ctx is None:
                self._w("program not running")
            else:
                for k in sorted(self.ctx.vars):
                    self._w(f"  {k}: {self._what(self.ctx.vars[k])}")
        elif c in ("p", "print", "w", "whatis") and args:
            found, v = self._lookup(args[0])
            if not found:
                self._w(f"variable {args[0]} not defined")
            else:
                self._w(self._what(v) if c in ("w", "whatis") else self._show(v))
        else:
            self._w(f"unknown command: {cmd}")

    @staticmethod
    def _what(v):
        if isinstance(v, torch.Tensor):
            fmt = "sparse" if v.layout != torch.strided else "dense"
            return f"matrix[{v.dtype}] {v.shape[0]}x{v.shape[1]} ({fmt}, {v.device})"
        if hasattr(v, "columns") and hasattr(v, "schema"):
            return f"frame {v.shape[0]}x{v.shape[1]}"
        if type(v).__name__ == "CompressedMatrix":
            return f"matrix {v.shape[0]}x{v.shape[1]} (compressed)"
        return f"scalar[{type(v).__name__}] {v!r}"

    @staticmethod
    def _show(v, k=6):
        if isinstance(v, torch.Tensor):
            d = v.to_dense() if v.layout != torch.strided else v
            d = d[:k, :k].double().cpu().numpy()
            return "\n".join(" ".join(f"{x:.4g}" for x in row) for row in d)
        return repr(v)
