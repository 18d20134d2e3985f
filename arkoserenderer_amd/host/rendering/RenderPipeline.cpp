#include "RenderPipeline.h"

#include "core/Logging.h"

const RenderPipelineNode::ExecuteCallback RenderPipelineNode::NullExecuteCallback = [](const AppState&, CommandList&, UploadBuffer&) {};

namespace ark {
int& errorCounter()
{
    static int n = 0;
    return n;
}
const char* logLevelName(LogLevel l)
{
    switch (l) {
    case LogLevel::Verbose: return "verbose";
    case LogLevel::Info: return "info";
    case LogLevel::Warning: return "warning";
    case LogLevel::Error: return "error";
    default: return "fatal";
    }
}
} // namespace ark

RenderPipelineNode& RenderPipeline::addNode(std::unique_ptr<RenderPipelineNode>&& node)
{
    ARKOSE_ASSERT(m_nodeContexts.empty()); // all nodes are added before construction
    m_ownedNodes.emplace_back(std::move(node));
    return *m_ownedNodes.back();
}

void RenderPipeline::constructAll(Registry& registry)
{
    m_nodeContexts.clear();
    for (auto& node : m_ownedNodes) {
        registry.setCurrentNode(node->name());
        auto cb = node->construct(*m_scene, registry);
        m_nodeContexts.push_back({ node.get(), std::move(cb) });
        registry.m_allNodeNames.push_back(node->name());
    }
    registry.setCurrentNode(std::nullopt);
}

void RenderPipeline::forEachNodeInResolvedOrder(const std::function<void(RenderPipelineNode&, const RenderPipelineNode::ExecuteCallback&)>& callback) const
{
    ARKOSE_ASSERT(!m_nodeContexts.empty());
    for (const NodeContext& c : m_nodeContexts) callback(*c.node, c.executeCallback);
}

void RenderPipeline::executeFrame(const AppState& appState, HipBackend& backend) const
{
    CommandList cmdList(backend.stream());
    UploadBuffer upload;
    forEachNodeInResolvedOrder([&](RenderPipelineNode&, const RenderPipelineNode::ExecuteCallback& cb) { cb(appState, cmdList, upload); });
}
