// proc_obj.cpp -- write the C5 procedural heightfield (ceres_proc_mesh) as OBJ
// text: n*n "v x y z" lines (float32 values printed with %.9g, which round-trips exactly) and
// 2(n-1)^2 "f a b c" lines in ceres_proc_mesh's triangle order, so parsing the file yields
// exactly ceres_proc_mesh's triangles and normals.   usage: proc_obj N out.obj
#include <cmath>
#include <cstdio>
#include <cstdlib>

int main(int argc, char** argv) {
    if (argc != 3) { std::fprintf(stderr, "usage: proc_obj N out.obj\n"); return 2; }
    const int n = std::atoi(argv[1]);
    if (n < 2) return 2;
    std::FILE* f = std::fopen(argv[2], "wb");
    if (!f) return 1;
    static char buf[1 << 20];
    std::setvbuf(f, buf, _IOFBF, sizeof buf);
    std::fprintf(f, "# C5 heightfield %d x %d\n", n, n);
    for (int j = 0; j < n; ++j)
        for (int i = 0; i < n; ++i) {
            const double x = double(i) / double(n - 1), y = double(j) / double(n - 1);
            const double z = 0.05 * (std::sin(40.0 * x) + std::cos(37.0 * y)) + 0.01 * std::sin(400.0 * x + 300.0 * y);
            std::fprintf(f, "v %.9g %.9g %.9g\n", double(float(x)), double(float(y)), double(float(z)));
        }
    for (int j = 0; j + 1 < n; ++j)
        for (int i = 0; i + 1 < n; ++i) {
            const long a = long(j) * n + i + 1, b = a + 1, c = a + n + 1, d = a + n;
            std::fprintf(f, "f %ld %ld %ld\nf %ld %ld %ld\n", a, b, c, a, c, d);
        }
    return std::fclose(f) == 0 ? 0 : 1;
}
