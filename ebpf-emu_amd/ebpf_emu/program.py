"""Program / batch API: load once, run(packets) -> verdicts on the GPU.

This is the batched form of the reference's per-packet composite
    Emu::default(); mmu = Mmu{1 KiB, packet at [0,len)}; regs r1=0,r2=len,r10=512; emu.run();
    verdict = emu.state.regs[0]                    (main.rs:14-43, emu.rs:30-45,452-458)
over device-resident frames. Device memory and streams come from PyTorch (plumbing only); the
work is one launch of the gfx950 kernel in libebpfemu.so per batch.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

from . import _lib
from .ins import DecodeError, _decoded, load_image


@dataclass
class BatchResult:
    verdict: object = None   # torch.uint8 [n]
    r0: object = None        # torch.int64 [n] (u64 bits)
    status: object = None    # torch.uint8 [n]
    counters: object = None  # torch.int64 [8] (u64 bits), accumulated
    mem: object = None       # torch.uint8 [n, mem_size]
    regs: object = None      # torch.int64 [n, 11]
    fp: object = None        # torch.int32 [n, 64] (u32 bits): final frame stacks, bottom first
    fp_len: object = None    # torch.uint8 [n]: their depths


def _ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


class Program:
    """A loaded eBPF program (ebpf_prog_load). Immutable; shareable across devices."""

    def __init__(self, image: bytes):
        self._h = load_image(bytes(image))
        self.image = bytes(image)

    @classmethod
    def from_hex(cls, hx: str) -> "Program":
        L = _lib.lib()
        h = ctypes.c_void_p()
        bad = ctypes.c_size_t(0)
        rc = L.ebpf_prog_load_hex(hx.encode(), ctypes.byref(h), ctypes.byref(bad))
        if rc != 0:
            raise DecodeError(rc, bad.value)
        self = cls.__new__(cls)
        self._h = h
        self.image = None
        return self

    def __len__(self) -> int:
        return _lib.lib().ebpf_prog_len(self._h)

    @property
    def tier(self) -> int:
        return _lib.lib().ebpf_prog_tier(self._h)

    @property
    def forward_only(self) -> bool:
        """True when batches run on the forward-jump fast path (max_steps >= len(self))."""
        return bool(_lib.lib().ebpf_prog_forward_only(self._h))

    @property
    def stack_window(self) -> int:
        """Memory tier 0.5: bytes of the stack window kept in registers (ebpf_prog_stack_window),
        0 when the program is not a stack-window program."""
        return _lib.lib().ebpf_prog_stack_window(self._h)

    def compile(self) -> bool:
        """Compile to gfx950 code now (ebpf_prog_compile): True if this is a compiled program
        (tier 0 or the stack / store tiers, <= EBPF_MAX_COMPILED_UOPS = 4096 micro-ops), False if it
        runs interpreted."""
        rc = _lib.lib().ebpf_prog_compile(self._h)
        if rc < 0:
            raise _lib.EbpfError(rc, "ebpf_prog_compile")
        return rc == 1

    def jit_asm(self, variant: int = 1) -> str:
        """The compiled program's assembly (variant 1: the main.rs register layout, 0: with
        init_regs)."""
        L = _lib.lib()
        n = ctypes.c_size_t(0)
        rc = L.ebpf_prog_jit_asm(self._h, variant, None, 0, ctypes.byref(n))
        if rc:
            raise _lib.EbpfError(rc, "ebpf_prog_jit_asm")
        buf = ctypes.create_string_buffer(n.value + 1)
        L.ebpf_prog_jit_asm(self._h, variant, buf, n.value + 1, ctypes.byref(n))
        return buf.value.decode()

    @property
    def jit_error(self) -> str:
        """Why the program is not (wholly) compiled (ebpf_prog_jit_error): the compiler's or the
        assembler's message, or why it is not a program the compiler takes; "" if compiled."""
        L = _lib.lib()
        n = ctypes.c_size_t(0)
        rc = L.ebpf_prog_jit_error(self._h, None, 0, ctypes.byref(n))
        if rc:
            raise _lib.EbpfError(rc, "ebpf_prog_jit_error")
        buf = ctypes.create_string_buffer(n.value + 1)
        L.ebpf_prog_jit_error(self._h, buf, n.value + 1, ctypes.byref(n))
        return buf.value.decode()

    @property
    def window_bytes(self) -> int:
        """Bytes of each packet's 64-byte header window the compiled fixed-slot kernel DMAs
        (jit.cpp window_chunks: the 16-byte chunks its constant-address loads and stores reach;
        all 64 with a register-address load)."""
        import re

        try:
            a = self.jit_asm(1)
        except _lib.EbpfError:
            return 64
        m = re.search(r"s_mov_b32 exec_lo, (0x[0-9a-f]+)\ns_mov_b32 exec_hi, (0x[0-9a-f]+)", a)
        if not m:
            return 64
        lanes = bin(int(m.group(1), 16)).count("1") + bin(int(m.group(2), 16)).count("1")
        return lanes  # (16 lanes per chunk, 16 bytes each, per 16 packets: 1 byte per lane)

    @property
    def store_mode(self) -> bool:
        """Register-address stores into the packet (host.cpp analyze_stack, StackPlan::any_dyn):
        the compiled var kernel with its header window in LDS and the deopt pass."""
        return _lib.lib().ebpf_prog_store_mode(self._h) > 0

    @property
    def store_mode_no_deopt(self) -> bool:
        """Store mode with no lane able to deoptimize on the var tile loop (jit.cpp
        store_mode_no_deopt): main.rs-layout batches run without the deopt pass."""
        return _lib.lib().ebpf_prog_store_mode(self._h) == 2

    @property
    def promoted(self) -> bool:
        """A stack-window loop program with its 8-byte slots promoted to registers (host.cpp
        promote_slots): production batches run that tier-0 program (compiled variant 4) on the
        loop kernels, EBPF_KERNEL_JIT_LOOP."""
        try:
            return bool(self.jit_asm(4))
        except _lib.EbpfError:
            return False

    def jit_loop_kernel(self) -> str:
        """The template kernel holding this program's compiled loop code (EBPF_KERNEL_JIT_LOOP
        names either): "ebpf_tile_jit_loop_deep" when the loop program went to the deep kernel
        (cooperative byte sums, or a deeper refill prefetch), else "ebpf_tile_jit_loop". (For a
        promoted stack program: its promoted program's kernel.)"""
        a = self.jit_asm(4 if self.promoted else 2)
        at = 0
        for ln in a.splitlines(keepends=True):
            at += len(ln)
            if ln.startswith("; JIT N=") and " loops=1" in ln and " stack=1" not in ln:
                if "not this program's kernel" not in a[at:at + 80]:
                    return "ebpf_tile_jit_loop_deep" if " deep=1" in ln else "ebpf_tile_jit_loop"
        return "ebpf_tile_jit_loop"

    @property
    def instructions(self):
        return _decoded(self._h)

    def close(self) -> None:
        if getattr(self, "_h", None):
            _lib.lib().ebpf_prog_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def upload(self, device: int) -> None:
        rc = _lib.lib().ebpf_prog_upload(self._h, device)
        if rc:
            raise _lib.EbpfError(rc, "ebpf_prog_upload")

    def make_batch(self, frames, n: int | None = None, stride: int = 0, offsets=None, lens=None,
                   mem_size: int = _lib.DEFAULT_MEM, r10: int = _lib.DEFAULT_R10,
                   max_steps: int = _lib.DEFAULT_STEPS, init_regs=None,
                   workspace=None, generic: bool = False, xdp_md: bool = False,
                   no_jit: bool = False, init_fp=None) -> _lib.Batch:
        b = _lib.Batch()
        _lib.lib().ebpf_batch_init(ctypes.byref(b))
        if n is None:
            n = offsets.numel() if offsets is not None else frames.numel() // max(stride, 1)
        b.frames = frames.data_ptr()
        b.offsets = offsets.data_ptr() if offsets is not None else None
        b.lens = lens.data_ptr() if lens is not None else None
        b.stride = stride
        b.n = n
        b.mem_size = mem_size
        b.r10 = r10 & ((1 << 64) - 1)
        b.max_steps = max_steps
        b.init_regs = init_regs.data_ptr() if init_regs is not None else None
        if init_fp is not None and init_fp.numel():
            b.init_fp = init_fp.data_ptr()
            b.init_fp_len = init_fp.numel()
        b.flags = ((_lib.BATCH_GENERIC if generic else 0) | (_lib.BATCH_XDP_MD if xdp_md else 0) |
                   (_lib.BATCH_NO_JIT if no_jit else 0))
        if workspace is not None:
            b.workspace = workspace.data_ptr()
            b.workspace_bytes = workspace.numel() * workspace.element_size()
        return b

    def batch_kernel(self, batch: _lib.Batch, out: _lib.BatchOut | None = None,
                     device: int = 0) -> int:
        """The EBPF_KERNEL_* id of the kernel ebpf_run_batch runs for `batch` and `out` on
        `device` (ebpf_batch_kernel; _lib.KERNEL_NAMES[id] names it)."""
        o = out if out is not None else _lib.BatchOut()
        rc = _lib.lib().ebpf_batch_kernel(self._h, ctypes.byref(batch), ctypes.byref(o), device)
        if rc < 0:
            raise _lib.EbpfError(rc, "ebpf_batch_kernel")
        return rc

    def batch_staged(self, batch: _lib.Batch, out: _lib.BatchOut | None = None,
                     device: int = 0) -> bool:
        """Whether ebpf_run_batch stages this xdp_md batch's images before the program's kernel
        (ebpf_batch_staged); False when it runs in place or is not an xdp_md batch."""
        o = out if out is not None else _lib.BatchOut()
        rc = _lib.lib().ebpf_batch_staged(self._h, ctypes.byref(batch), ctypes.byref(o), device)
        if rc < 0:
            raise _lib.EbpfError(rc, "ebpf_batch_staged")
        return rc == 1

    def workspace_bytes(self, batch: _lib.Batch, device: int) -> int:
        return int(_lib.lib().ebpf_workspace_bytes(self._h, ctypes.byref(batch), device))

    def launch(self, batch: _lib.Batch, out: _lib.BatchOut, stream=None) -> None:
        """Raw asynchronous launch on `stream` (a torch.cuda.Stream or None = current)."""
        import torch

        s = stream if stream is not None else torch.cuda.current_stream()
        rc = _lib.lib().ebpf_run_batch(self._h, ctypes.byref(batch), ctypes.byref(out),
                                       ctypes.c_void_p(s.cuda_stream))
        if rc:
            raise _lib.EbpfError(rc, "ebpf_run_batch")

    def run(self, frames, n: int | None = None, stride: int = 0, offsets=None, lens=None,
            mem_size: int = _lib.DEFAULT_MEM, r10: int = _lib.DEFAULT_R10,
            max_steps: int = _lib.DEFAULT_STEPS, init_regs=None, verdict: bool = True,
            r0: bool = False, status: bool = False, counters=None, mem: bool = False,
            regs: bool = False, stream=None, generic: bool = False,
            xdp_md: bool = False, no_jit: bool = False, init_fp=None,
            fp: bool = False) -> BatchResult:
        """Run the program over a device-resident batch; returns device tensors.

        frames: torch.uint8 CUDA tensor. Layout: packet i at frames[i*stride:] (stride layout,
        len = lens[i] or stride) or at frames[offsets[i]:] (offsets: torch.int32 / uint32 bits,
        lens: torch.int16/uint16 bits). counters: an optional torch.int64 [8] tensor to add to.
        generic: run on the general interpreter even if the forward-jump fast path applies.
        no_jit: run a compiled program (compile()) on the tile interpreter instead.
        init_fp: an optional device int32 tensor, the initial frame stack (Emu.fp, emu.rs:26) of
        every packet, bottom first; fp: return the final frame stacks (res.fp, res.fp_len).
        xdp_md: the xdp_md calling convention (EBPF_BATCH_XDP_MD): each image is
        [u32 data = 8][u32 data_end = 8 + len][packet], r1 = 0 the ctx, r2 = 8 + len.
        """
        import torch

        dev = frames.device
        b = self.make_batch(frames, n, stride, offsets, lens, mem_size, r10, max_steps, init_regs,
                            generic=generic, xdp_md=xdp_md, no_jit=no_jit, init_fp=init_fp)
        n = b.n
        res = BatchResult()
        if verdict:
            res.verdict = torch.empty(n, dtype=torch.uint8, device=dev)
        if r0:
            res.r0 = torch.empty(n, dtype=torch.int64, device=dev)
        if status:
            res.status = torch.empty(n, dtype=torch.uint8, device=dev)
        if mem:
            res.mem = torch.empty((n, mem_size), dtype=torch.uint8, device=dev)
        if regs:
            res.regs = torch.empty((n, 11), dtype=torch.int64, device=dev)
        if fp:
            res.fp = torch.zeros((n, _lib.MAX_CALL_DEPTH), dtype=torch.int32, device=dev)
            res.fp_len = torch.empty(n, dtype=torch.uint8, device=dev)
        res.counters = counters
        out = _lib.BatchOut()
        out.verdict = res.verdict.data_ptr() if verdict else None
        out.r0 = res.r0.data_ptr() if r0 else None
        out.status = res.status.data_ptr() if status else None
        out.counters = counters.data_ptr() if counters is not None else None
        out.mem = res.mem.data_ptr() if mem else None
        out.regs = res.regs.data_ptr() if regs else None
        out.fp = res.fp.data_ptr() if fp else None
        out.fp_len = res.fp_len.data_ptr() if fp else None
        with torch.cuda.device(dev):
            self.launch(b, out, stream)
        return res


def u64(t):
    """torch.int64 tensor of u64 bit patterns -> list of Python ints in [0, 2**64)."""
    return [int(v) & ((1 << 64) - 1) for v in t.tolist()]
