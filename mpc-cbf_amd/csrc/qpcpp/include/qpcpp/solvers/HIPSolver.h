// HIPSolver.h — qpcpp::Solver<T> backend that solves a qpcpp::Problem on the MI355X through the
// C ABI (include/mpccbf.h, mpccbf_qp_solve_dense). Drop-in for CPLEXSolver<T>
// (qpcpp/include/qpcpp/solvers/CPLEX.h:19-24): same solve(Problem&) -> SolveStatus contract
// (Solver.h:27-37), solution written back through Variable::set_solution_value only when the
// status is OPTIMAL (Solver.h:33-35), never throws for solver failures (ERROR instead).
//
// Header-only and written against the reference's public qpcpp API only (variables(),
// linear_constraints(), cost_function() getters), so the reference keeps its own Problem
// implementation; a maintainer adds this header and re-points the solver alias, e.g.
// ConnectivityIMPCCBF.h:36 `using CPLEXSolver = qpcpp::CPLEXSolver<T>` -> HIPSolver<T>.
//
// Flattening follows what CPLEXSolver::solve hands to CPLEX (CPLEX.cpp:52-147):
//   - variable i = position in problem.variables() (forward_list order),
//   - objective sum_{i<=j} q_ij x_i x_j + sum c_i x_i + const  ->  x^T H x + c^T x + c0 with
//     H_ii = q_ii, H_ij = H_ji = q_ij / 2 (no 1/2 factor: Problem.cpp:101-116 convention),
//   - rows min <= a^T x <= max, variable bounds min <= x_i <= max; numeric_limits lowest()/max()
//     are infinite (|v| >= 1e300 in the C ABI).
#pragma once

#include <qpcpp/Problem.h>
#include <qpcpp/solvers/Solver.h>

#include <cstddef>
#include <unordered_map>
#include <vector>

#include "mpccbf.h"

namespace qpcpp {

struct FlatQP {
    int n = 0, m = 0;
    std::vector<double> H, c, A, lo, hi, vlo, vhi;
    double c0 = 0.0;
};

template <typename T>
class HIPSolver : public Solver<T> {
  public:
    using Base = Solver<T>;
    using Problem = typename Base::Problem;
    using Variable = qpcpp::Variable<T>;

    // Flattened CPLEX form of `problem`; `order` receives the variable of every column.
    static FlatQP flatten(Problem& problem, std::vector<const Variable*>& order) {
        FlatQP f;
        order.clear();
        for (const Variable& v : problem.variables()) order.push_back(&v);
        const int n = (int)order.size();
        f.n = n;
        f.H.assign((size_t)n * n, 0.0);
        f.c.assign(n, 0.0);
        f.vlo.resize(n);
        f.vhi.resize(n);
        auto* cost = problem.cost_function();
        for (int i = 0; i < n; i++) {
            f.vlo[i] = (double)order[i]->min();
            f.vhi[i] = (double)order[i]->max();
            f.c[i] = (double)cost->getLinearCoefficient(order[i]);
            for (int j = i; j < n; j++) {
                const double q = (double)cost->getQuadraticCoefficient(order[i], order[j]);
                if (q == 0.0) continue;
                if (i == j) {
                    f.H[(size_t)i * n + i] += q;
                } else {
                    f.H[(size_t)i * n + j] += 0.5 * q;
                    f.H[(size_t)j * n + i] += 0.5 * q;
                }
            }
        }
        f.c0 = (double)cost->constant();
        for (const auto& row : problem.linear_constraints()) {
            for (int j = 0; j < n; j++) f.A.push_back((double)row.getCoefficient(order[j]));
            f.lo.push_back((double)row.min());
            f.hi.push_back((double)row.max());
            f.m++;
        }
        return f;
    }

    SolveStatus solve(Problem& problem) override {
        std::vector<const Variable*> order;
        const FlatQP f = flatten(problem, order);
        mpccbf_dense_qp qp;
        qp.n = f.n;
        qp.m = f.m;
        qp.H = f.H.data();
        qp.c = f.c.data();
        qp.c0 = f.c0;
        qp.A = f.m ? f.A.data() : nullptr;
        qp.lo = f.m ? f.lo.data() : nullptr;
        qp.hi = f.m ? f.hi.data() : nullptr;
        qp.vlo = f.vlo.data();
        qp.vhi = f.vhi.data();
        std::vector<double> x(f.n, 0.0);
        double obj = 0.0;
        int32_t st = MPCCBF_ERROR;
        if (f.n == 0 || mpccbf_qp_solve_dense(&qp, x.data(), &obj, &st) != MPCCBF_OK)
            return SolveStatus::ERROR;  // mpccbf_last_error() has the reason
        const SolveStatus status = static_cast<SolveStatus>(st);  // same enumerator order
        if (status == SolveStatus::OPTIMAL || status == SolveStatus::FEASIBLE) {
            for (int i = 0; i < f.n; i++)
                const_cast<Variable*>(order[i])->set_solution_value(static_cast<T>(x[i]));
        }
        last_objective_ = obj;
        return status;
    }

    // Objective of the last OPTIMAL solve (CPLEX getObjValue, CPLEX.cpp:144-146).
    double last_objective() const { return last_objective_; }

  private:
    double last_objective_ = 0.0;
};

}  // namespace qpcpp
