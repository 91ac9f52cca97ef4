// qpcpp/solvers/Solver.h — header-only host mirror of the reference solver interface
// (workspace/lib/qpcpp/include/qpcpp/solvers/Solver.h:13-37, src/solvers/Solver.cpp:4-28):
// the SolveStatus enumerators in the same order (their indices are the MPCCBF_* status codes of
// include/mpccbf.h) and the abstract Solver<T>::solve(Problem&).
#pragma once

#include <string>

#include <qpcpp/Problem.h>

namespace qpcpp {

enum class SolveStatus { OPTIMAL, FEASIBLE, UNBOUNDED, INFEASIBLE, ERROR, UNKNOWN, INFEASIBLEORUNBOUNDED };

inline std::string SolveStatusToStr(SolveStatus s) {
    static const char* const names[] = {"OPTIMAL", "FEASIBLE", "UNBOUNDED", "INFEASIBLE",
                                        "ERROR",   "UNKNOWN",  "INFEASIBLEORUNBOUNDED"};
    const int i = static_cast<int>(s);
    return (i >= 0 && i < 7) ? names[i] : "";
}

template <typename T>
class Solver {
  public:
    using Problem = qpcpp::Problem<T>;
    virtual ~Solver() = default;
    // Sets Variable::solution_value only when the status is OPTIMAL or FEASIBLE.
    virtual SolveStatus solve(Problem& problem) = 0;
};

}  // namespace qpcpp
