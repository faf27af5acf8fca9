// skirt_host_write_descriptors (include/skirt_host.h): a canonical dump of the engine's input descriptors
// (SkirtGridDesc, SkirtMediaDesc, SkirtSourceDesc, SkirtInstrDesc), so that two producers of them can be
// compared field by field without a device: the .ski driver (skirt_sim_describe) and the maintainer binding
// that extracts them from SKIRT's own set-up simulation items (integration/GpuPhotonEngine.cpp,
// tests/test_binding_describe.py).
//
// Format, one record per field, appended to the file: "<name> <type> <count>\n" then count raw
// little-endian values (type d: double, i: int32, b: int8). Array lengths follow skirt_mcrt.h.
#include <cstdio>
#include <string>

#include "../../../include/skirt_host.h"

namespace {

struct Writer {
    FILE* f;
    void rec(const std::string& name, char type, size_t size, const void* p, size_t n) {
        std::fprintf(f, "%s %c %zu\n", name.c_str(), type, n);
        if (n && p) std::fwrite(p, size, n, f);
    }
    void d(const std::string& name, const double* p, size_t n) { rec(name, 'd', sizeof(double), p, p ? n : 0); }
    void i(const std::string& name, const int* p, size_t n) { rec(name, 'i', sizeof(int), p, p ? n : 0); }
    void b(const std::string& name, const signed char* p, size_t n) { rec(name, 'b', 1, p, p ? n : 0); }
    void d1(const std::string& name, double v) { d(name, &v, 1); }
    void i1(const std::string& name, int v) { i(name, &v, 1); }
};

void writeGrid(Writer& w, const SkirtGridDesc& g) {
    w.i1("grid.kind", g.kind);
    w.i1("grid.ncells", g.ncells);
    if (g.kind == SKIRT_GRID_CARTESIAN) {
        w.i1("grid.nx", g.nx);
        w.i1("grid.ny", g.ny);
        w.i1("grid.nz", g.nz);
        w.d("grid.xv", g.xv, (size_t)g.nx + 1);
        w.d("grid.yv", g.yv, (size_t)g.ny + 1);
        w.d("grid.zv", g.zv, (size_t)g.nz + 1);
    } else if (g.kind == SKIRT_GRID_OCTREE) {
        const size_t n = (size_t)g.nnodes;
        w.i1("grid.nnodes", g.nnodes);
        w.d("grid.box", g.box, 6 * n);
        w.i("grid.first_child", g.first_child, n);
        w.i("grid.cellnumber", g.cellnumber, n);
        w.i("grid.nbr_offset", g.nbr_offset, 6 * n + 1);
        w.i("grid.nbr_list", g.nbr_list, g.nbr_offset ? (size_t)g.nbr_offset[6 * n] : 0);
        w.b("grid.split_dir", g.split_dir, n);
        w.d1("grid.eps", g.eps);
        w.i1("grid.search", g.search);
    } else {
        const size_t nc = (size_t)g.ncells, nb3 = (size_t)g.nblocks * g.nblocks * g.nblocks;
        w.d("grid.site", g.site, 3 * nc);
        w.i("grid.cell_nbr_offset", g.cell_nbr_offset, nc + 1);
        w.i("grid.cell_nbr_list", g.cell_nbr_list, g.cell_nbr_offset ? (size_t)g.cell_nbr_offset[nc] : 0);
        w.d("grid.cell_bbox", g.cell_bbox, 6 * nc);
        w.d("grid.extent", g.extent, 6);
        w.d1("grid.eps", g.eps);
        w.i1("grid.nblocks", g.nblocks);
        w.i("grid.block_offset", g.block_offset, nb3 + 1);
        w.i("grid.block_list", g.block_list, g.block_offset ? (size_t)g.block_offset[nb3] : 0);
    }
}

void writeMedia(Writer& w, const SkirtMediaDesc& m) {
    const size_t t = (size_t)m.ncomp * m.nlambda;
    w.i1("media.ncells", m.ncells);
    w.i1("media.ncomp", m.ncomp);
    w.i1("media.nlambda", m.nlambda);
    w.d("media.rho", m.rho, (size_t)m.ncells * m.ncomp);
    w.d("media.kext", m.kext, t);
    w.d("media.ksca", m.ksca, t);
    w.d("media.albedo", m.albedo, t);
    w.d("media.g", m.g, t);
}

void writeSources(Writer& w, const SkirtSourceDesc& s) {
    const size_t nc = (size_t)s.ncomp, nl = (size_t)s.nlambda;
    w.i1("sources.ncomp", s.ncomp);
    w.i1("sources.nlambda", s.nlambda);
    w.i("sources.geom_kind", s.geom_kind, nc);
    w.d("sources.geom_param", s.geom_param, 8 * nc);
    w.d("sources.lum", s.lum, nc * nl);
    w.d("sources.lumtot", s.lumtot, nl);
    w.d("sources.cdf", s.cdf, nl * (nc + 1));
    w.d1("sources.emission_bias", s.emission_bias);
    w.d("sources.geom_table", s.geom_table, 202 * nc);
}

void writeInstruments(Writer& w, const SkirtInstrDesc* d, int n) {
    w.i1("instruments.n", n);
    for (int k = 0; k < n; k++) {
        const SkirtInstrDesc& x = d[k];
        const std::string p = "instrument" + std::to_string(k) + ".";
        w.i1(p + "kind", x.kind);
        w.i1(p + "nx", x.nx);
        w.i1(p + "ny", x.ny);
        w.i1(p + "scattering_levels", x.scattering_levels);
        w.d(p + "kobs", x.kobs, 3);
        const double v[10] = {x.sinphi, x.cosphi, x.sintheta, x.costheta, x.sinpa, x.cospa,
                              x.xpmin, x.xpsiz, x.ypmin, x.ypsiz};
        const char* names[10] = {"sinphi", "cosphi", "sintheta", "costheta", "sinpa", "cospa",
                                 "xpmin", "xpsiz", "ypmin", "ypsiz"};
        for (int q = 0; q < 10; q++) w.d1(p + names[q], v[q]);
    }
}

}  // namespace

extern "C" int skirt_host_write_descriptors(const char* path, const SkirtGridDesc* grid, const SkirtMediaDesc* media,
                                            const SkirtSourceDesc* sources, const SkirtInstrDesc* instr, int ninstr) {
    if (!path) return SKIRT_ERR_ARG;
    FILE* f = std::fopen(path, "ab");
    if (!f) return SKIRT_ERR_ARG;
    Writer w{f};
    if (grid) writeGrid(w, *grid);
    if (media) writeMedia(w, *media);
    if (sources) writeSources(w, *sources);
    if (ninstr >= 0) writeInstruments(w, instr, ninstr);
    const bool ok = std::fclose(f) == 0;
    return ok ? SKIRT_OK : SKIRT_ERR_ARG;
}
