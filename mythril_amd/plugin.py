"""LASER plugin that switches the prune point to the batched GPU pre-filter.

Reference interface mirrored (duck-typed — mythril is not importable here):

  LaserPlugin.initialize(symbolic_vm)       laser/ethereum/plugins/plugin.py:4-23
  LaserPluginLoader.load(plugin)            laser/ethereum/plugins/plugin_loader.py:24-31
  PluginFactory.build_*_plugin()            laser/ethereum/plugins/plugin_factory.py:4-41

The reference has no hook at the prune filter (svm.py:251-255: every
successor's ``constraints.is_possible`` is read one at a time, each a fresh z3
check).  The plugin therefore wraps two LaserEVM methods instead of adding a
hook:

* ``execute_state`` — after the instruction ran, the successors' constraint
  sets go through ONE ``batch_is_possible`` call (one GPU batch, then the
  reference's 100 ms fallback for every state without a witness).  The
  results land in each ``Constraints._is_possible`` cache, so the unchanged
  filter in ``exec`` only reads cached bits.  A child inherits its parent's
  witness as the first candidate (a JUMPI child differs from its parent by
  one constraint).
* ``exec`` (only with ``window > 1``) — a copy of svm.py:220-264 that pulls up
  to ``window`` states from the strategy, executes them, and prunes all their
  successors in one batch.  For the breadth-first strategy the work-list order
  is exactly the sequential one (successors are appended behind every state
  already queued, strategy/basic.py:50-61), so BFS -- the CLI's default strategy
  (interfaces/cli.py:405-410) -- gets ``window = BFS_WINDOW`` unless the caller
  picks one.  Every other strategy (DFS pops the newest state, basic.py:36-47; the
  random ones draw from the whole list, basic.py:64-92) would see a different work
  list with a window, so ``initialize`` forces ``window = 1`` for them.  Only
  BoundedLoopsStrategy is looked through (via ``super_strategy``): its pick reads the
  popped state alone.  CoverageStrategy's pick depends on coverage, which changes as
  states run, so under it the window is 1.

Everything the GPU cannot prove satisfiable reaches the fallback solver with
the reference's own arguments, so the pruning decision is the reference's
whenever the fallback answers sat/unsat.
"""
from __future__ import annotations

import logging
from datetime import datetime, timedelta
from typing import Callable, List, Optional, Sequence

from . import solver as SV

log = logging.getLogger(__name__)


def _constraints_of(global_state):
    return global_state.world_state.constraints


# Wrappers whose pick depends only on the popped state itself, so picking a window of states
# before any of them runs gives the sequential order.  BoundedLoopsStrategy reads the state's
# own JumpdestCountAnnotation (strategy/extensions/bounded_loops.py:27-141).  CoverageStrategy
# (plugins/implementations/coverage/coverage_strategy.py:8-37) is NOT one: it picks the first
# state at an uncovered instruction, and coverage changes as states execute.
_ORDER_PRESERVING_WRAPPERS = frozenset({"BoundedLoopsStrategy"})


def is_breadth_first(strategy) -> bool:
    """Is the strategy BreadthFirstSearchStrategy, under wrappers that keep its order?"""
    seen = 0
    while strategy is not None and seen < 16:
        name = type(strategy).__name__
        if name == "BreadthFirstSearchStrategy":
            return True
        if name not in _ORDER_PRESERVING_WRAPPERS:
            return False
        strategy = getattr(strategy, "super_strategy", None)
        seen += 1
    return False


class GpuPrefilterPlugin:
    """The toggle: loading it routes LASER's prune point through the GPU.

    window=None: BFS_WINDOW states per batch under breadth-first search, 1 otherwise;
    an explicit window > 1 is honoured only under breadth-first search."""

    BFS_WINDOW = 16

    def __init__(self, window: Optional[int] = None, batch: Callable[[Sequence], List[bool]] = SV.batch_is_possible,
                 constraints_of: Callable = _constraints_of):
        if window is not None and window < 1:
            raise ValueError("window must be >= 1")
        self.requested_window = window
        self.window = window or 1
        self._batch = batch
        self._constraints_of = constraints_of
        self.batches = 0
        self.states_checked = 0

    def __repr__(self):
        return f"GpuPrefilterPlugin(window={self.window})"

    # plugins/plugin.py:18-23
    def initialize(self, symbolic_vm) -> None:
        SV.enable_gpu(True)
        if is_breadth_first(getattr(symbolic_vm, "strategy", None)):
            self.window = self.requested_window or self.BFS_WINDOW
        else:
            if (self.requested_window or 1) > 1:
                log.warning("GPU pre-filter: window=%d needs breadth-first search; using window=1",
                            self.requested_window)
            self.window = 1
        orig_execute = symbolic_vm.execute_state

        def execute_state(global_state):
            new_states, op_code = orig_execute(global_state)
            if self.window == 1:
                self.prune_batch([global_state], [new_states])
            return new_states, op_code

        symbolic_vm.execute_state = execute_state
        if self.window > 1:
            symbolic_vm.exec = lambda create=False, track_gas=False: self._exec(symbolic_vm, create, track_gas)

    def prune_batch(self, parents: Sequence, successor_lists: Sequence[Sequence]) -> None:
        """Fill every successor's is_possible cache with one batched query."""
        todo = []
        for parent, succ in zip(parents, successor_lists):
            pw = getattr(self._constraints_of(parent), "witness", None)
            for s in succ:
                c = self._constraints_of(s)
                if getattr(c, "_is_possible", True) is None:
                    if getattr(c, "witness", None) is None and pw is not None:
                        c.witness = pw
                    todo.append(c)
        if todo:
            self._batch(todo)
            self.batches += 1
            self.states_checked += len(todo)

    # svm.py:220-264 with a batch window over the strategy
    def _exec(self, vm, create: bool = False, track_gas: bool = False):
        final_states: List = []
        it = iter(vm.strategy)
        while True:
            window = []
            for _ in range(self.window):
                try:
                    window.append(next(it))
                except StopIteration:
                    break
            if not window:
                break
            executed = []
            stopped = None
            for gs in window:
                # svm.py:229-244: the timeout is checked before every state; the first state
                # not executed is returned behind the final states
                if self._timed_out(vm, create):
                    stopped = gs
                    break
                try:
                    new_states, op_code = vm.execute_state(gs)
                except NotImplementedError:
                    log.debug("Encountered unimplemented instruction")
                    continue
                executed.append((gs, new_states, op_code))
            self.prune_batch([e[0] for e in executed], [e[1] for e in executed])
            for gs, new_states, op_code in executed:
                new_states = [s for s in new_states if self._constraints_of(s).is_possible]
                vm.manage_cfg(op_code, new_states)
                if new_states:
                    vm.work_list += new_states
                elif track_gas:
                    final_states.append(gs)
                vm.total_states += len(new_states)
            if stopped is not None:
                log.debug("Hit timeout, returning.")
                return final_states + [stopped] if track_gas else None
        return final_states if track_gas else None

    @staticmethod
    def _timed_out(vm, create: bool) -> bool:
        now = datetime.now()
        if getattr(vm, "create_timeout", None) and create and vm.time + timedelta(seconds=vm.create_timeout) <= now:
            return True
        if getattr(vm, "execution_timeout", None) and not create and \
                vm.time + timedelta(seconds=vm.execution_timeout) <= now:
            return True
        return False


class PluginFactory:
    """plugin_factory.py:4-41 — one more builder next to the reference's."""

    @staticmethod
    def build_gpu_prefilter_plugin(window: Optional[int] = None) -> GpuPrefilterPlugin:
        return GpuPrefilterPlugin(window=window)


class LaserPluginLoader:
    """plugin_loader.py:10-37 (same behaviour: initialize, then remember)."""

    def __init__(self, symbolic_vm) -> None:
        self.symbolic_vm = symbolic_vm
        self.laser_plugins: List = []

    def load(self, laser_plugin) -> None:
        log.info("Loading plugin: %s", laser_plugin)
        laser_plugin.initialize(self.symbolic_vm)
        self.laser_plugins.append(laser_plugin)

    def is_enabled(self, laser_plugin) -> bool:
        return laser_plugin in self.laser_plugins


def disable() -> Optional[bool]:
    """Turn the GPU stage off again (the reference path: every query to the fallback)."""
    SV.enable_gpu(False)
    return None
