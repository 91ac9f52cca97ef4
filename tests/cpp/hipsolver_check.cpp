// hipsolver_check.cpp — drives qpcpp::HIPSolver<double> (csrc/qpcpp/include/qpcpp/solvers/) on
// qpcpp::Problem instances built exactly as the reference's callers build them (the host mirror
// in csrc/qpcpp/include). Test infrastructure, used by tests/test_qpcpp_adapter.py.
//
//   hipsolver_check flatten   print the flattened CPLEX form of the test problems (no GPU)
//   hipsolver_check solve     solve them on the GPU, print status / solution / objective
//
// Problem 0 is CPLEXTest::SolveSimpleQP (qpcpp/tests/CPLEXTest.cpp:28-56). Problem 1 adds an
// equality, a cross term, a constant, variable bounds and a ranged row.
#include <cstdio>
#include <cstring>
#include <limits>
#include <vector>

#include <qpcpp/solvers/HIPSolver.h>

using P = qpcpp::Problem<double>;

static void build(int which, P& problem, std::vector<qpcpp::Variable<double>*>& vars) {
    vars.clear();
    if (which == 0) {
        auto* x = problem.addVariable();
        auto* y = problem.addVariable();
        vars = {x, y};
        auto* cost = problem.cost_function();
        cost->addQuadraticTerm(x, x, 1.0);
        cost->addQuadraticTerm(y, y, 1.0);
        auto* row = problem.addLinearConstraint(1.0, std::numeric_limits<double>::max());
        row->setCoefficient(x, 1.0);
        row->setCoefficient(y, 1.0);
    } else {
        // min (x-1)^2 + (y-2)^2 + x z + z^2 + 3   s.t.  x + y + z = 1,  -1 <= x - z <= 0.5,
        //     0 <= x <= 0.25, z >= -2
        auto* x = problem.addVariable(0.0, 0.25);
        auto* y = problem.addVariable();
        auto* z = problem.addVariable(-2.0);
        vars = {x, y, z};
        auto* cost = problem.cost_function();
        cost->addQuadraticTerm(x, x, 1.0);
        cost->addLinearTerm(x, -2.0);
        cost->addQuadraticTerm(y, y, 1.0);
        cost->addLinearTerm(y, -4.0);
        cost->addQuadraticTerm(z, x, 1.0);  // reversed pair: stored once for (x, z)
        cost->addQuadraticTerm(z, z, 1.0);
        cost->add_constant(5.0 + 3.0);
        auto* eq = problem.addLinearConstraint(1.0, 1.0);
        eq->setCoefficient(x, 1.0);
        eq->setCoefficient(y, 1.0);
        eq->setCoefficient(z, 1.0);
        auto* rg = problem.addLinearConstraint(-1.0, 0.5);
        rg->setCoefficient(x, 1.0);
        rg->setCoefficient(z, -1.0);
    }
}

static void print_vec(const char* key, const std::vector<double>& v) {
    std::printf("\"%s\": [", key);
    for (size_t i = 0; i < v.size(); i++) std::printf("%s%.17g", i ? ", " : "", v[i]);
    std::printf("]");
}

int main(int argc, char** argv) {
    const bool solve = argc > 1 && std::strcmp(argv[1], "solve") == 0;
    for (int which = 0; which < 2; which++) {
        P problem;
        std::vector<qpcpp::Variable<double>*> vars;
        build(which, problem, vars);
        std::printf("{\"problem\": %d, ", which);
        if (!solve) {
            std::vector<const qpcpp::Variable<double>*> order;
            const qpcpp::FlatQP f = qpcpp::HIPSolver<double>::flatten(problem, order);
            std::vector<double> col;  // column of each variable in creation order
            for (auto* v : vars)
                for (size_t j = 0; j < order.size(); j++)
                    if (order[j] == v) col.push_back((double)j);
            std::printf("\"n\": %d, \"m\": %d, \"c0\": %.17g, ", f.n, f.m, f.c0);
            print_vec("col", col), std::printf(", ");
            print_vec("H", f.H), std::printf(", ");
            print_vec("c", f.c), std::printf(", ");
            print_vec("A", f.A), std::printf(", ");
            print_vec("lo", f.lo), std::printf(", ");
            print_vec("hi", f.hi), std::printf(", ");
            print_vec("vlo", f.vlo), std::printf(", ");
            print_vec("vhi", f.vhi);
        } else {
            qpcpp::HIPSolver<double> solver;
            const qpcpp::SolveStatus st = solver.solve(problem);
            std::vector<double> x;
            for (auto* v : vars) x.push_back(st == qpcpp::SolveStatus::OPTIMAL ? v->solution_value() : 0.0);
            std::printf("\"status\": \"%s\", \"obj\": %.17g, ", qpcpp::SolveStatusToStr(st).c_str(),
                        solver.last_objective());
            print_vec("x", x);
            if (st == qpcpp::SolveStatus::ERROR) std::printf(", \"error\": \"%s\"", mpccbf_last_error());
        }
        std::printf("}\n");
    }
    return 0;
}
