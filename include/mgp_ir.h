/*
 * mgp_ir.h — constraint-DAG node format and bytecode encoding of the
 * Mythril GPU pre-filter (MI355X / gfx950).
 *
 * A state's path constraints (laser.smt Bool / BitVec expressions, reference
 * mythril/laser/smt/{bitvec,bitvec_helper,bool,function}.py) are handed over
 * as a topologically ordered node list (mgp_node).  The last node is the
 * root and must be Bool.  Semantics are z3 / SMT-LIB bit-vector semantics,
 * NOT EVM semantics:
 *   UDIV x/0 = 2^w-1, UREM x%0 = x, SDIV x/0 = (x<0 ? 1 : 2^w-1),
 *   SREM sign follows dividend, SMOD sign follows divisor, x%0 = x,
 *   SHL/LSHR by >= w -> 0, ASHR by >= w -> sign fill.
 *
 * The host lowering (mgp_lower) turns each node list into the flat bytecode
 * below, which the HIP kernel evaluates for every candidate assignment.
 *
 * This header is plain C, shared by the HIP kernels, the C++ host runtime
 * and (read-only) by the oracle as the interface definition.
 */
#ifndef MGP_IR_H
#define MGP_IR_H

#include <stdint.h>

#define MGP_MAX_WIDTH 256   /* widest bit-vector a kernel slot holds        */
#define MGP_MAX_WIDE 2048   /* widest DAG value (split into <= 256-bit pieces) */

/* Wide values (MGP_MAX_WIDTH < width <= MGP_MAX_WIDE): the reference builds
 * 512-bit mapping preimages Concat(key, slot) for keccak256_512 and its
 * inverse (keccak_function_manager.py:56-69,122-146), 257-bit overflow sums
 * and 776-bit calldata hashes.  In a DAG they are held as ceil(width/256)
 * consecutive entries, low 256 bits first:
 *   VAR    variables p0, p0+1, ...        CONST  pool entries p0, p0+1, ...
 *   UFAPP / UFINV with a wide result: fresh variables p1, p1+1, ...
 * CONCAT, EXTRACT, ZEXT, ITE, EQ, UF arguments/results, ADD / SUB (carry chain
 * between pieces: the 257-bit BVAddNoOverflow expansions), MUL (128-bit limb
 * schoolbook: the 512-bit BVMulNoOverflow expansion), AND / OR / XOR / NOT and
 * the unsigned compares ULT / ULE / UGT / UGE may touch a wide value; the
 * lowering splits it into pieces and emits narrow code only.  Any other op on a
 * wide value (division, shifts, signed compares) makes the state
 * MGP_ST_UNSUPPORTED. */
#define MGP_LIMBS 8         /* 8 x u32 little-endian limbs per 256-bit value */

/* ---------------------------------------------------------------- opcodes */
enum mgp_op {
  /* leaves (DAG only) */
  MGP_OP_VAR = 1,     /* p0 = candidate variable index, width = var width   */
  MGP_OP_CONST = 2,   /* p0 = constant-pool index (8 u32 limbs)             */
  MGP_OP_TRUE = 3,
  MGP_OP_FALSE = 4,

  /* BV x BV -> BV (all operands of the result width) */
  MGP_OP_ADD = 8,     /* bvadd   bitvec.py:63            */
  MGP_OP_SUB = 9,     /* bvsub   bitvec.py:76            */
  MGP_OP_MUL = 10,    /* bvmul   bitvec.py:89            */
  MGP_OP_UDIV = 11,   /* bvudiv  bitvec_helper.py:145    */
  MGP_OP_UREM = 12,   /* bvurem  bitvec_helper.py:125    */
  MGP_OP_SDIV = 13,   /* bvsdiv  bitvec.py:96 (__truediv__) */
  MGP_OP_SREM = 14,   /* bvsrem  bitvec_helper.py:135    */
  MGP_OP_SMOD = 15,   /* bvsmod  (z3 BitVecRef.__mod__)   */
  MGP_OP_AND = 16,    /* bvand   bitvec.py:105           */
  MGP_OP_OR = 17,     /* bvor    bitvec.py:117           */
  MGP_OP_XOR = 18,    /* bvxor   bitvec.py:129           */
  MGP_OP_NOT = 19,    /* bvnot (unary)                   */
  MGP_OP_NEG = 20,    /* bvneg (unary)                   */
  MGP_OP_SHL = 21,    /* bvshl   bitvec.py:232           */
  MGP_OP_LSHR = 22,   /* bvlshr  bitvec_helper.py:21     */
  MGP_OP_ASHR = 23,   /* bvashr  bitvec.py:240 (>>)      */
  MGP_OP_EXTRACT = 24,/* a; p0 = hi, p1 = lo  bitvec_helper.py:115 */
  MGP_OP_CONCAT = 25, /* a (high) , b (low)   bitvec_helper.py:93  */
  MGP_OP_ZEXT = 26,   /* a zero-extended to width                   */
  MGP_OP_SEXT = 27,   /* a sign-extended to width                   */
  MGP_OP_ITE = 28,    /* a = Bool cond, b = then, c = else  bitvec_helper.py:25 */

  /* BV x BV -> Bool (operands share one width) */
  MGP_OP_EQ = 40,     /* =      bitvec.py:183 (_padded_operation done by builder) */
  MGP_OP_ULT = 41,    /* bvult  bitvec_helper.py:63 */
  MGP_OP_ULE = 42,    /* bvule  (Or(ULT, ==))  bitvec_helper.py:73 */
  MGP_OP_UGT = 43,    /* bvugt  bitvec_helper.py:43 */
  MGP_OP_UGE = 44,    /* bvuge  bitvec_helper.py:53 */
  MGP_OP_SLT = 45,    /* bvslt  bitvec.py:138 (<)  */
  MGP_OP_SLE = 46,    /* bvsle  bitvec.py:160 (<=) */
  MGP_OP_SGT = 47,    /* bvsgt  bitvec.py:149 (>)  */
  MGP_OP_SGE = 48,    /* bvsge  bitvec.py:171 (>=) */
  MGP_OP_UADD_NOOVF = 49, /* BVAddNoOverflow(a,b,False) bitvec_helper.py:168 */
  MGP_OP_UMUL_NOOVF = 50, /* BVMulNoOverflow(a,b,False) bitvec_helper.py:183 */
  MGP_OP_USUB_NOUDF = 51, /* BVSubNoUnderflow(a,b,False) bitvec_helper.py:199 */

  /* Bool -> Bool */
  MGP_OP_BAND = 60,   /* bool.py:87  (binary; n-ary is chained) */
  MGP_OP_BOR = 61,    /* bool.py:106 */
  MGP_OP_BXOR = 62,   /* bool.py:99  */
  MGP_OP_BNOT = 63,   /* bool.py:120 */
  MGP_OP_BITE = 64,   /* a = cond, b = then, c = else (Bool) */
  MGP_OP_BEQ = 65,    /* Bool == Bool (bool.py:50) */

  /* uninterpreted functions (DAG only; lowered to ITE chains = Ackermann
   * expansion with a lazily built, always-consistent interpretation)
   *   UFAPP  f(a):     value of the first earlier f-app whose argument equals a,
   *                    else candidate variable p1 (fresh value).
   *   UFINV  f^-1(a):  value of the first earlier f^-1-app whose argument equals a,
   *                    else the argument of the first earlier f-app whose value
   *                    equals a, else candidate variable p1.
   * p0 = function id (the forward function for UFINV).  keccak_function_manager.py:56-69 */
  MGP_OP_UFAPP = 70,
  MGP_OP_UFINV = 71,

  /* bytecode only */
  MGP_OP_MOV = 80,    /* dst = a masked to width */
  /* one step of an f-application chain (UFAPP above; a Select over a Store chain, a
   * calldata byte table): result = (a == b) ? c : ACC, the else value being the
   * accumulator (the previous BV instruction's result); a, b, c never name ACC */
  MGP_OP_EQSEL = 81,
  MGP_OP_RET = 90     /* root = Bool operand a   */
};

/* ------------------------------------------------------------- DAG nodes */
typedef struct mgp_node {
  uint8_t op;        /* enum mgp_op                          */
  uint8_t flags;     /* reserved, 0                           */
  uint16_t width;    /* result width in bits (1 for Bool)     */
  int32_t a, b, c;   /* operand node indices (< own index), -1 = none */
  uint32_t p0, p1;   /* op parameters (see enum)              */
} mgp_node;          /* 24 bytes */

/* --------------------------------------------------------------- bytecode
 * Per state, 16-byte aligned (offsets in u32 words, multiple of 4):
 *   header  : w0 = n_ins, w1 = n_consts, w2 = n_slots (BV slots used, spill
 *             slots included), w3 = status (MGP_ST_*) | max_var << 8
 *   n_ins   x 4 words  instructions
 *   n_consts x 8 words constants (little-endian u32 limbs)
 *
 * instruction words:
 *   w0 = op | (width-1) << 8 | dst << 16 | flags << 24
 *   w1 = operand A | operand B << 16
 *   w2 = operand C | imm << 16
 *   w3 = 0 (reserved)
 * For Bool-producing ops dst is a bool bit; for BV-producing ops dst is a BV
 * slot (written only if MGP_INS_STORE) and the result always lands in the
 * accumulator (ACC operand of the next instruction).
 * For compare ops `width` is the OPERAND width.
 * imm: EXTRACT lo bit; CONCAT low-part width; SEXT source width.
 */
#define MGP_HDR_WORDS 4
#define MGP_INS_WORDS 4
#define MGP_INS_STORE 0x1u

/* BV slots 0..MGP_LDS_SLOTS-1 live in per-lane LDS.  A slot s >= MGP_LDS_SLOTS is a
 * SPILL slot: it lives in the evaluating lane's own candidate row, at variable index
 * MGP_SPILL_BASE(max_var) + (s - MGP_LDS_SLOTS), where max_var = header w3 >> 8 (one
 * past the highest variable the program reads), so a spill never overlaps a variable
 * the program reads.  Every spill slot is written before it is read.  A program with
 * spill slots therefore needs a candidate block of at least MGP_PROG_VARS(header)
 * variables per state; the rows past the state's own variables are scratch (the
 * gfx950 interpreter keeps up to 31 slots in LDS and may use one more spill row, which
 * MGP_PROG_VARS includes).  Slot numbers of a spilling program are ordered by access
 * count, so the most used values stay in LDS. */
#define MGP_LDS_SLOTS 32u
#define MGP_MAX_SLOTS 4095u  /* BV destination: 8 bits in word 0 (bits 16..23), the high bits in word 3 */
#define MGP_SPILL_BASE(max_var) ((max_var) > 8u ? (max_var) : 8u)
#define MGP_PROG_VARS(h)                                                                        \
  ((h)[2] >= MGP_LDS_SLOTS ? MGP_SPILL_BASE((h)[3] >> 8) + (h)[2] - MGP_LDS_SLOTS + 1u : ((h)[3] >> 8))
/* live Bool values a program keeps in bits; past it the lowering demotes the Bool
 * with the farthest next use to a 1-bit BV value (ITE(b, 1, 0), re-tested by EQ at
 * each reader), which can spill like any BV value (= the gfx950 interpreter's 17
 * allocatable Bool registers) */
#ifndef MGP_BOOL_LIVE
#define MGP_BOOL_LIVE 17u
#endif

/* BV operand (16 bits): kind in bits 15:14, index in 13:0 */
#define MGP_K_SLOT 0u
#define MGP_K_CONST 1u
#define MGP_K_ACC 2u
#define MGP_K_VAR 3u
#define MGP_OPND(kind, idx) ((uint32_t)(((kind) << 14) | ((idx)&0x3FFFu)))

/* Bool operands are plain bit indices.  Bits 62/63 hold constant false/true. */
#define MGP_BOOL_BITS 64
#define MGP_BOOL_FALSE 62
#define MGP_BOOL_TRUE 63
#define MGP_BOOL_ALLOC 62   /* bits 0..61 are allocatable */

/* per-state status (header w3 and lowering status output) */
#define MGP_ST_OK 0
#define MGP_ST_UNSUPPORTED 1   /* arithmetic on a wide value, too many live values, unknown op */

/* first-SAT sentinels */
#define MGP_NO_SAT (-1)
#define MGP_UNDECIDED (-2)
/* an evaluation wave left no valid result for the state (internal inconsistency; never
 * expected — reported instead of reading a candidate outside the batch) */
#define MGP_EVAL_FAULT (-3)

#endif /* MGP_IR_H */
