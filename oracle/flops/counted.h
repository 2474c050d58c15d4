/* ORACLE / TEST INFRASTRUCTURE ONLY: the instrumented build of the oracle
   (flops/Makefile) compiles mjsub.c / ilqr_ora.c as C++ with mjtNum = ora_f,
   a double that counts every fp64 add/sub, mul, div, sqrt and comparison it
   takes part in (SURVEY.md §8d "Algorithmic flops": an instrumented build of
   the CPU restatement).  Arithmetic is unchanged: each operator applies the
   same IEEE operation to the wrapped doubles. */
#pragma once
#include <cmath>

struct ora_flop_counts {
  unsigned long long add, mul, div, sqrt, cmp, trans;
};
extern "C" ora_flop_counts ora_flops;

struct ora_f {
  double v;
  ora_f() = default;
  constexpr ora_f(double x) : v(x) {}
  explicit operator double() const { return v; }
  explicit operator bool() const { return v != 0; }
  ora_f& operator+=(ora_f b) { ora_flops.add++; v += b.v; return *this; }
  ora_f& operator-=(ora_f b) { ora_flops.add++; v -= b.v; return *this; }
  ora_f& operator*=(ora_f b) { ora_flops.mul++; v *= b.v; return *this; }
  ora_f& operator/=(ora_f b) { ora_flops.div++; v /= b.v; return *this; }
  ora_f operator-() const { return ora_f(-v); }
  ora_f operator+() const { return *this; }
};

#define ORA_BIN(op, cnt)                                                                  \
  inline ora_f operator op(ora_f a, ora_f b) { ora_flops.cnt++; return ora_f(a.v op b.v); } \
  inline ora_f operator op(ora_f a, double b) { ora_flops.cnt++; return ora_f(a.v op b); }  \
  inline ora_f operator op(double a, ora_f b) { ora_flops.cnt++; return ora_f(a op b.v); }  \
  inline ora_f operator op(ora_f a, int b) { ora_flops.cnt++; return ora_f(a.v op b); }     \
  inline ora_f operator op(int a, ora_f b) { ora_flops.cnt++; return ora_f(a op b.v); }
ORA_BIN(+, add)
ORA_BIN(-, add)
ORA_BIN(*, mul)
ORA_BIN(/, div)
#undef ORA_BIN
#define ORA_CMP(op)                                                                        \
  inline bool operator op(ora_f a, ora_f b) { ora_flops.cmp++; return a.v op b.v; }         \
  inline bool operator op(ora_f a, double b) { ora_flops.cmp++; return a.v op b; }          \
  inline bool operator op(double a, ora_f b) { ora_flops.cmp++; return a op b.v; }          \
  inline bool operator op(ora_f a, int b) { ora_flops.cmp++; return a.v op b; }             \
  inline bool operator op(int a, ora_f b) { ora_flops.cmp++; return a op b.v; }
ORA_CMP(<)
ORA_CMP(>)
ORA_CMP(<=)
ORA_CMP(>=)
ORA_CMP(==)
ORA_CMP(!=)
#undef ORA_CMP
inline ora_f sqrt(ora_f a) { ora_flops.sqrt++; return ora_f(std::sqrt(a.v)); }
inline ora_f fabs(ora_f a) { return ora_f(std::fabs(a.v)); }
inline ora_f floor(ora_f a) { return ora_f(std::floor(a.v)); }
#define ORA_MJTNUM ora_f
#define ORA_FLOP_TRANS() (ora_flops.trans++)
inline ora_f atan2(ora_f a, ora_f b) { ora_flops.trans++; return ora_f(std::atan2(a.v, b.v)); }
