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
#include <string>
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

// The bookkeeping tests of the reference's qpcpp/tests/ProblemTest.cpp:19-137, restated against the
// host mirror of qpcpp::Problem (csrc/qpcpp/include/qpcpp/Problem.h) that HIPSolver flattens. One
// JSON line per test: {"test": name, "ok": bool, "failed": [expectations that failed]}.
static int problem_tests() {
    using V = qpcpp::Variable<double>;
    int failures = 0;
    auto report = [&](const char* name, const std::vector<std::string>& failed) {
        std::printf("{\"test\": \"%s\", \"ok\": %s, \"failed\": [", name, failed.empty() ? "true" : "false");
        for (size_t i = 0; i < failed.size(); i++) std::printf("%s\"%s\"", i ? ", " : "", failed[i].c_str());
        std::printf("]}\n");
        failures += failed.empty() ? 0 : 1;
    };
#define EXPECT(cond) \
    if (!(cond)) f.push_back(#cond)
    {  // InitialProblemStateIsEmpty (:19-23)
        std::vector<std::string> f;
        P problem;
        EXPECT(problem.numVariables() == 0);
        EXPECT(problem.numLinearConstraints() == 0);
        report("InitialProblemStateIsEmpty", f);
    }
    {  // AddingVariablesIncreasesCount (:25-31)
        std::vector<std::string> f;
        P problem;
        problem.addVariable(-1.0, 1.0);
        EXPECT(problem.numVariables() == 1);
        problem.addVariable(-2.0, 2.0);
        EXPECT(problem.numVariables() == 2);
        report("AddingVariablesIncreasesCount", f);
    }
    {  // VariableMinMaxLimits (:33-43)
        std::vector<std::string> f;
        P problem;
        V* var = problem.addVariable(-1.5, 2.5);
        EXPECT(var->min() == -1.5);
        EXPECT(var->max() == 2.5);
        var->set_min(-3.0);
        var->set_max(4.0);
        EXPECT(var->min() == -3.0);
        EXPECT(var->max() == 4.0);
        report("VariableMinMaxLimits", f);
    }
    {  // HasVariableTest (:45-56)
        std::vector<std::string> f;
        P problem;
        V* var1 = problem.addVariable();
        V* var2 = problem.addVariable();
        EXPECT(problem.hasVariable(var1));
        EXPECT(problem.hasVariable(var2));
        P other_problem;
        V* other_var = other_problem.addVariable();
        EXPECT(!problem.hasVariable(other_var));
        report("HasVariableTest", f);
    }
    {  // VariableSolutionValueTest (:58-64)
        std::vector<std::string> f;
        P problem;
        V* var = problem.addVariable(-1.0, 1.0);
        var->set_solution_value(0.5);
        EXPECT(var->solution_value() == 0.5);
        report("VariableSolutionValueTest", f);
    }
    {  // AddingConstraintsIncreasesCount (:66-72)
        std::vector<std::string> f;
        P problem;
        problem.addLinearConstraint(-1.0, 1.0);
        EXPECT(problem.numLinearConstraints() == 1);
        problem.addLinearConstraint(-2.0, 2.0);
        EXPECT(problem.numLinearConstraints() == 2);
        report("AddingConstraintsIncreasesCount", f);
    }
    {  // ConstraintCoefficients (:74-85)
        std::vector<std::string> f;
        P problem;
        V* var1 = problem.addVariable();
        V* var2 = problem.addVariable();
        auto* constraint = problem.addLinearConstraint(0.0, 5.0);
        constraint->setCoefficient(var1, 2.0);
        constraint->setCoefficient(var2, 3.0);
        EXPECT(constraint->getCoefficient(var1) == 2.0);
        EXPECT(constraint->getCoefficient(var2) == 3.0);
        report("ConstraintCoefficients", f);
    }
    {  // ClearingConstraints (:87-95)
        std::vector<std::string> f;
        P problem;
        problem.addLinearConstraint();
        problem.addLinearConstraint();
        EXPECT(problem.numLinearConstraints() == 2);
        problem.clearLinearConstraints();
        EXPECT(problem.numLinearConstraints() == 0);
        report("ClearingConstraints", f);
    }
    {  // CostFunctionLinearTerms (:97-108)
        std::vector<std::string> f;
        P problem;
        V* var1 = problem.addVariable();
        V* var2 = problem.addVariable();
        auto* cost = problem.cost_function();
        cost->addLinearTerm(var1, 2.5);
        cost->addLinearTerm(var2, 3.5);
        EXPECT(cost->getLinearCoefficient(var1) == 2.5);
        EXPECT(cost->getLinearCoefficient(var2) == 3.5);
        report("CostFunctionLinearTerms", f);
    }
    {  // CostFunctionQuadraticTerms (:110-121)
        std::vector<std::string> f;
        P problem;
        V* var1 = problem.addVariable();
        V* var2 = problem.addVariable();
        auto* cost = problem.cost_function();
        cost->addQuadraticTerm(var1, var2, 2.5);
        EXPECT(cost->getQuadraticCoefficient(var1, var2) == 2.5);
        EXPECT(cost->getQuadraticCoefficient(var2, var1) == 2.5);  // symmetry
        report("CostFunctionQuadraticTerms", f);
    }
    {  // ResetProblem (:123-137)
        std::vector<std::string> f;
        P problem;
        V* var = problem.addVariable();
        problem.addLinearConstraint();
        auto* cost = problem.cost_function();
        cost->addLinearTerm(var, 1.0);
        EXPECT(problem.numLinearConstraints() == 1);
        EXPECT(cost->getLinearCoefficient(var) == 1.0);
        problem.resetProblem();
        EXPECT(problem.numLinearConstraints() == 0);
        EXPECT(cost->getLinearCoefficient(var) == 0.0);
        report("ResetProblem", f);
    }
#undef EXPECT
    return failures;
}

int main(int argc, char** argv) {
    if (argc > 1 && std::strcmp(argv[1], "problemtest") == 0) return problem_tests() == 0 ? 0 : 1;
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
