// The maintainer binding's data extraction, run without a device (tests/test_binding_describe.py, VERDICT r5
// item 6). Sets a .ski up with the reference's own classes -- XmlHierarchyCreator and Simulation::setup, as
// SkirtCommandLineHandler::doSimulation does (SKIRTmain/SkirtCommandLineHandler.cpp:259-348), on one thread
// like `skirt -t 1` -- then hands the set-up items to GpuPhotonEngine::describe and writes the descriptors
// it builds with skirt_host_write_descriptors. The test compares the file with skirt_sim_describe's for the
// same .ski: what the binding would upload inside SKIRT against what the .ski driver uploads.
//   describe file.ski out.bin outdir
// Built by integration/build_describe.sh from the reference objects of oracle/ref.mk (build container only).
#include <clocale>
#include <cstdio>

#include <QCoreApplication>
#include <QSharedPointer>

#include "DustSystem.hpp"
#include "FatalError.hpp"
#include "FilePaths.hpp"
#include "InstrumentSystem.hpp"
#include "Log.hpp"
#include "MonteCarloSimulation.hpp"
#include "ParallelFactory.hpp"
#include "PeerToPeerCommunicator.hpp"
#include "ProcessManager.hpp"
#include "RegisterSimulationItems.hpp"
#include "Simulation.hpp"
#include "StellarSystem.hpp"
#include "WavelengthGrid.hpp"
#include "XmlHierarchyCreator.hpp"

#include "GpuPhotonEngine.hpp"
#include "skirt_host.h"

namespace
{
    class FileSink : public GpuDescriptorSink
    {
    public:
        explicit FileSink(const char* path) : _path(path) {}
        void grid(const SkirtGridDesc& g) override { put(skirt_host_write_descriptors(_path, &g, 0, 0, 0, -1)); }
        void media(const SkirtMediaDesc& m) override { put(skirt_host_write_descriptors(_path, 0, &m, 0, 0, -1)); }
        void sources(const SkirtSourceDesc& s) override { put(skirt_host_write_descriptors(_path, 0, 0, &s, 0, -1)); }
        void instruments(const SkirtInstrDesc* d, int n) override
        {
            put(skirt_host_write_descriptors(_path, 0, 0, 0, d, n));
        }

    private:
        void put(int rc) { if (rc != SKIRT_OK) throw FATALERROR(QString("cannot write ") + _path); }
        const char* _path;
    };
}

int main(int argc, char** argv)
{
    if (argc != 4)
    {
        std::fprintf(stderr, "usage: describe file.ski out.bin outdir\n");
        return 2;
    }
    setlocale(LC_ALL, "C");
    ProcessManager::initialize(&argc, &argv);
    QCoreApplication app(argc, argv);
    RegisterSimulationItems::registerAll();
    try
    {
        XmlHierarchyCreator creator;
        QSharedPointer<Simulation> simulation(creator.createHierarchy<Simulation>(QString(argv[1])));
        simulation->filePaths()->setOutputPrefix("describe");
        simulation->filePaths()->setOutputPath(QString(argv[3]) + "/");
        simulation->parallelFactory()->setMaxThreadCount(1);
        simulation->communicator()->setup();
        simulation->log()->setLowestLevel(Log::Error);
        simulation->setup();

        if (FILE* f = std::fopen(argv[2], "wb")) std::fclose(f);  // the sink appends
        DustSystem* ds = nullptr;
        try { ds = simulation->find<DustSystem>(false); }
        catch (FatalError&) {}
        FileSink sink(argv[2]);
        GpuPhotonEngine::describe(simulation->find<WavelengthGrid>(), simulation->find<StellarSystem>(), ds,
                                  simulation->find<InstrumentSystem>(), sink);
    }
    catch (FatalError& error)
    {
        for (QString line : error.message()) std::fprintf(stderr, "%s\n", line.toLocal8Bit().constData());
        return 1;
    }
    ProcessManager::finalize();
    return 0;
}
