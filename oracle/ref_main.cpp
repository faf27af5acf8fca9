// main() of the reference binary built by oracle/ref.mk (test infrastructure only; see that file).
// The reference's own main (SKIRTmain/SkirtMain.cpp:18-47) includes a git_version.h that its qmake project
// generates; this one runs the same start-up sequence against the reference's own classes and reports a fixed
// version string instead. Nothing here changes what a simulation computes or writes.
#include <clocale>
#include <QCoreApplication>
#include "ProcessManager.hpp"
#include "RegisterSimulationItems.hpp"
#include "SignalHandler.hpp"
#include "SkirtCommandLineHandler.hpp"

int main(int argc, char** argv)
{
    setlocale(LC_ALL, "C");                      // SkirtMain.cpp:21 (sprintf in cfitsio)
    ProcessManager::initialize(&argc, &argv);    // no-op without BUILDING_WITH_MPI
    QCoreApplication app(argc, argv);
    app.setApplicationName("SKIRT");
    app.setApplicationVersion("v7.3 (oracle/ref.mk build)");
    SignalHandler::InstallSignalHandlers();
    RegisterSimulationItems::registerAll();
    SkirtCommandLineHandler handler(app.arguments());
    int status = handler.perform();
    ProcessManager::finalize();
    return status;
}
